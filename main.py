#!/usr/bin/env python3
"""Drop-in CLI for the hot path of genome-minimizer-2's main.py (main.py:62-147, :647-692).

Implemented modes, same flags and file layout as the reference:
  --mode training --preset v0..v3 [--epochs N]     run_single_experiment (main.py:449-493)
  --mode sample --model-path ..._vK.pt --genes-path essential_gene_positions.pkl
        [--num-samples N] [--sampling-mode default|focused] [--noise-level s]   run_sampling (:219-446)
Both route through the gfx950 kernels of libgm2.so (gm2 package); there is no CPU path.

  --mode convert-samples --genes-path masks.npy [--output-file ids.npy]   run_binary_converter (:617-645)
        (host-side; the consumer of the sampled masks, explore_data/binary_converter.py)
  --mode minimizer --genes-path ids.npy [--genome-path wild_type.gb] [--single-file | --output-file f.fasta]
        [--output-dir d] [--model-name m]   run_genome_minimizer (:528-614), the consumer of the gene
        lists (gm2/minimizer.py: interval-union host rewrite of minimizer/minimizer_2.py)
Modes outside the MI355X hot path (explore, preprocess, experiment)
exit with code 2 and a message. Data files are looked up under the project root as in
utils/directories.py:13-20 (default: $GM2_PROJECT_ROOT or the current directory; --project-root).
Return codes follow main.py:647-692: 0 success, 1 failure.

Multi-GPU (no reference equivalent; the reference is single-device, main.py:37):
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 main.py --mode training ...
runs strain-row data parallelism over RCCL (gm2/ddp.py): every rank trains its share of each batch,
rank 0 prints and saves the checkpoint (--sync-bn: BatchNorm over the global batch, gm2/ddp.py).
--mode sample shards the genomes: one broadcast seed, the same z on every rank, each rank decodes its
contiguous slice on its GPU, rank 0 gathers the packed masks and writes the files. Other modes run
on rank 0 only.

Additions (no reference equivalent): --precision bf16|f32 for the training GEMMs (sampling always
decodes in exact fp32), --mask-dtype float64|uint8|bits for the saved masks (the reference writes
float64 via `.astype(float)`, main.py:369-371 / extras.py:200-201; uint8 keeps 1e6-genome runs in
memory; bits = numpy packbits(bitorder='little') rows, 1/64 of float64, accepted by convert-samples),
--no-csv to skip the genes x samples CSV. Sampling keeps the masks packed on the GPU: genome sizes
and essential-gene counts are computed there (gm2/masks.py) and only the packed rows cross PCIe.
"""
import argparse
import os
import pickle
import sys
import traceback
from pathlib import Path

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "genome-minimizer-2_amd"))

MODES = ["training", "experiment", "minimizer", "explore", "preprocess", "sample", "convert-samples"]
IMPLEMENTED = ("training", "sample", "convert-samples", "minimizer")


def parse_arguments(argv=None):
    p = argparse.ArgumentParser(description="genome-minimizer-2 VAE hot path on MI355X")
    p.add_argument("--mode", choices=MODES, default="training")
    p.add_argument("--preset", choices=["v0", "v1", "v2", "v3"], default="v3")
    p.add_argument("--epochs", type=int, default=None)
    p.add_argument("--model-path", type=str)
    p.add_argument("--genes-path", type=str)
    p.add_argument("--output-file", type=str)
    p.add_argument("--num-samples", type=int, default=1)
    p.add_argument("--sampling-mode", choices=["default", "focused"], default="default")
    p.add_argument("--noise-level", type=float, default=0.1)
    p.add_argument("--project-root", type=str, default=os.environ.get("GM2_PROJECT_ROOT", os.getcwd()))
    p.add_argument("--precision", choices=["bf16", "f32"], default="bf16")
    p.add_argument("--grad-exchange", choices=["f32", "bf16"], default=None,
                   help="torchrun / DDP only: dtype of the big weight-gradient all-reduce (default f32)")
    p.add_argument("--sync-bn", action="store_true",
                   help="torchrun / DDP only: train-mode BatchNorm over the global batch (SyncBN)")
    p.add_argument("--mask-dtype", choices=["float64", "uint8", "bits"], default="float64")
    p.add_argument("--no-csv", action="store_true")
    p.add_argument("--genome-path", type=str, default=None,
                   help="GenBank genome (default: <project root>/data/wild_type_sequence.gb)")
    p.add_argument("--output-dir", type=str, default="./minimized_genomes")
    p.add_argument("--single-file", action="store_true")
    p.add_argument("--model-name", type=str, default="default")
    return p.parse_args(argv)


def data_paths(root):
    """utils/directories.py:13-20."""
    d = os.path.join(root, "data")
    return {"Main Dataset": os.path.join(d, "F4_complete_presence_absence.csv"),
            "Phylogroups": os.path.join(d, "accessionID_phylogroup_BD.csv"),
            "Essential Genes": os.path.join(d, "essential_genes.csv")}


def check_data_availability(root):
    """main.py:149-170."""
    missing = [f"{k}: {v}" for k, v in data_paths(root).items() if not os.path.exists(v)]
    if missing:
        print("✗  Missing required data files:")
        for m in missing:
            print(f"   - {m}")
        return False
    print("✓ All required data files found")
    return True


PRECISION_NOTE = {
    "bf16": "bf16 GEMM operands, fp32 accumulation; fp32 master weights, BatchNorm, losses and Adam "
            "(--precision f32: the reference's fp32 arithmetic)",
    "f32": "fp32 throughout (the reference's arithmetic)",
}


def _precision(args):
    from gm2 import native
    return native.GM2_F32 if args.precision == "f32" else native.GM2_BF16


def run_single_experiment(args):
    """main.py:449-493: preset config, optional epoch override, run the experiment."""
    from gm2.experiments import PRESETS, IntegratedExperimentRunner
    config = PRESETS[args.preset]()
    if args.epochs:
        config.n_epochs = args.epochs
    print(f"\n{'=' * 80}\nRunning {config.experiment_name} experiment")
    print(f"Hidden dim: {config.hidden_dim}, Latent dim: {config.latent_dim}")
    print(f"Epochs: {config.n_epochs}, Trainer: {config.trainer_version}")
    # (not in the reference's header: its arithmetic is fp32 throughout; this build's default is
    # bf16 GEMMs -- pass --precision f32 for the reference's arithmetic)
    print(f"Precision: {PRECISION_NOTE[args.precision]}\n{'=' * 80}")
    paths = data_paths(args.project_root)
    runner = IntegratedExperimentRunner(config, project_root=args.project_root, precision=_precision(args),
                                        dataset_csv=paths["Main Dataset"], phylogroups_csv=paths["Phylogroups"])
    results = runner.run_complete_experiment()
    print(f"\n{config.experiment_name.upper()} COMPLETED!")
    return results


def detect_version(model_path):
    """main.py:292-304: preset from the checkpoint file name."""
    name = Path(model_path).name.lower()
    for v in ("v0", "v1", "v2", "v3"):
        if v in name:
            return v
    return None


def focused_z(model, latent_dim, num_samples, noise_level, device):
    """main.py:351-370: 100 default samples, the one with fewest genes, then its output-space
    nearest sample's z (the same index); returns z* + noise_level * N(0, I) [num_samples, L]."""
    import numpy as np
    import torch
    from gm2.extras import sample_from_model
    binary_temp, cont_temp, z_temp = sample_from_model(model, latent_dim, 100, device)
    min_ones_index = np.argmin(binary_temp.sum(axis=1))
    dist = np.linalg.norm(cont_temp - cont_temp[min_ones_index], axis=1)
    closest = np.argmin(dist)
    z_star = z_temp[closest].unsqueeze(0)
    noise = torch.randn(num_samples, latent_dim, device=device) * noise_level
    return z_star + noise


def focused_samples(model, latent_dim, num_samples, noise_level, device):
    """(u8 mask [N, G] on the device, z) of focused sampling."""
    z = focused_z(model, latent_dim, num_samples, noise_level, device)
    mask, _ = model.decode_mask(z)
    return mask, z


def run_sampling(args):
    """main.py:219-446 without the plots / PCA (out of scope): load the checkpoint, decode in fp32,
    threshold, count essential genes, save masks (.npy) and the genes x samples CSV."""
    import numpy as np
    import torch
    from gm2.data import load_and_validate_data
    from gm2.experiments import PRESETS
    from gm2.extras import count_essential_genes, load_model, write_samples_to_dataframe

    if not args.model_path:
        print("✗ Model path required for sampling mode")
        return False
    if not os.path.exists(args.model_path):
        print(f"✗ Model file not found: {args.model_path}")
        return False
    if not args.genes_path or not os.path.exists(args.genes_path):
        print(f"✗ Model file not found: {args.genes_path}. Run preprocessing first.")
        return False
    paths = data_paths(args.project_root)
    _, merged, _ = load_and_validate_data(paths["Main Dataset"], paths["Phylogroups"])
    all_genes = merged.columns[:-1]
    input_dim = len(all_genes)
    print(f"Detected input dimension: {input_dim}")
    with open(args.genes_path, "rb") as f:
        # the user's own preprocessing output, read the way the reference reads it (main.py:273-274)
        essential_gene_positions = pickle.load(f)
    version = detect_version(args.model_path)
    if version is None:
        print("✗ Could not detect version")
        return False
    config = PRESETS[version]()
    out_dir = Path(args.project_root) / "models" / f"{version}_model" / "sampling_results"
    out_dir.mkdir(parents=True, exist_ok=True)
    device = torch.device("cuda", torch.cuda.current_device())
    model = load_model(input_dim, config.hidden_dim, config.latent_dim, args.model_path)
    print(f"- Architecture: {input_dim} -> {config.hidden_dim} -> {config.latent_dim}")
    print(f"- Samples: {args.num_samples}\n- Mode: {args.sampling_mode}\n- Output: {out_dir}")
    from gm2.ddp import gather_rows, get_dist, rank_slice, rank_world, shared_seed
    dist = get_dist()
    rank, world = rank_world(dist)
    if dist is not None:
        # every rank draws the same z from one broadcast seed (the reference's z is one unseeded
        # draw of the global generator, extras.py:197) and decodes its contiguous slice
        torch.cuda.manual_seed(shared_seed(dist))
    if args.sampling_mode == "default":
        with torch.no_grad():
            z = torch.randn(args.num_samples, config.latent_dim, device=device)  # extras.py:197
    else:
        z = focused_z(model, config.latent_dim, args.num_samples, args.noise_level, device)
    lo, hi = rank_slice(args.num_samples, rank, world)
    st0 = model.decode_stats()
    packed, _ = model.decode_bits(z[lo:hi])   # masks stay on the GPU, 8 genes per byte
    st = {k: v - st0[k] for k, v in model.decode_stats().items()}
    # (this rank's decode: output-layer tiles per path and the certified band)
    print(f"- Decode (rank {rank}): {st['single_tiles']} bf16 / {st['split_tiles']} bf16x3 / {st['exact_tiles']} fp32 "
          f"output tiles; "
          f"{st['band_elements']} band logits recomputed in fp64, {st['band_flips']} bits changed"
          + (f"; {st['band_overflow']} past the list, their {st['overflow_tiles']} blocks recomputed whole in fp64"
             if st["band_overflow"] else ""))
    if dist is not None:
        # the ranks' packed slices -> the full set (rank 0 writes the reference's files)
        from gm2.masks import PackedMasks
        packed = PackedMasks(gather_rows(dist, packed.bits, args.num_samples), packed.G)
        if rank != 0:
            return True
    sizes = packed.row_sizes()                # binary.sum(axis=1)
    ess = count_essential_genes(packed, essential_gene_positions)  # on the device
    print(f"\n✓ Sampling Results:\n- Generated samples: {packed.n}")
    print(f"- Median genome size: {np.median(sizes):.0f} genes")
    print(f"- Genome size range: {np.min(sizes):.0f} - {np.max(sizes):.0f}")
    print(f"- Median essential genes: {np.median(ess):.0f}")
    print(f"- Essential range: {np.min(ess):.0f} - {np.max(ess):.0f}")
    if args.mask_dtype == "bits":
        out = packed.to_host()
    else:
        out = packed.unpack(np.float64 if args.mask_dtype == "float64" else np.uint8)
    np.save(out_dir / f"{config.trainer_version}_binary_samples_{args.sampling_mode}.npy", out)
    if not args.no_csv:
        rows = out if args.mask_dtype != "bits" else packed.unpack(np.uint8)
        write_samples_to_dataframe(rows, all_genes, f"{out_dir}/{config.trainer_version}_data_full_samples_df.csv")
    print(f"\n✓ SAMPLING COMPLETE!\n- Results saved to: {out_dir}")
    return True


def run_binary_converter(args):
    """main.py:617-645: gene columns from the dataset CSV, masks -> gene-id lists, then the
    essential-gene fill (explore_data/binary_converter.py)."""
    import pandas as pd
    from gm2.binary_converter import check_essential_genes, load_files, masks_to_gene_lists
    if not args.genes_path:
        print("✗ --genes-path is required in convert-samples mode (input masks .npy)")
        return False
    if not os.path.exists(args.genes_path):
        print(f"✗ Input masks file not found: {args.genes_path}")
        return False
    out_path = args.output_file or "seq_out.npy"
    paths = data_paths(args.project_root)
    large = pd.read_csv(paths["Main Dataset"], index_col=0)
    cols = large.drop(index=["Lineage"], errors="ignore").transpose().columns
    masks_to_gene_lists(masks_npy_path=args.genes_path, cols=cols, out_ids_npy=out_path)
    essential_set, id_lists = load_files(paths["Essential Genes"], out_path)
    filled = check_essential_genes(essential_set, id_lists, out_path)
    print(f"✓ Binary conversion complete\n- Gene lists: {out_path}\n- Gene lists (essentials filled): {filled}")
    return True


def run_genome_minimizer(args):
    """main.py:528-614 (same checks, messages and output layout)."""
    from gm2.minimizer import process_multiple_genomes_multiple_files, process_multiple_genomes_single_file
    print("\n" + "=" * 80 + "\nGENOME MINIMIZER RUN\n" + "=" * 80)
    genome_path = args.genome_path or os.path.join(args.project_root, "data", "wild_type_sequence.gb")
    if not os.path.exists(genome_path):
        print(f"✗ Genome file not found: {genome_path}")
        return None
    if not args.genes_path:
        print("✗ Genes path required for genome minimizer")
        return None
    if not os.path.exists(args.genes_path):
        print(f"✗ Genes file not found: {args.genes_path}")
        return None
    print(f"\n{'=' * 80}\nProcessing genome: {Path(genome_path).name}\nUsing genes from: {Path(args.genes_path).name}"
          f"\nModel name: {args.model_name}\n{'=' * 80}")
    try:
        if args.output_file:
            output_dir, output_filename = Path(args.output_file).parent, Path(args.output_file).name
        elif args.single_file:
            output_dir, output_filename = Path(args.output_dir), f"minimized_genomes_{args.model_name}.fasta"
        else:
            output_dir, output_filename = Path(args.output_dir), None
        output_dir.mkdir(parents=True, exist_ok=True)
        print(f"✓ Created output directory: {output_dir}")
        if args.single_file or args.output_file:
            output_file = output_dir / output_filename
            print(f"Generating single FASTA file: {output_file}")
            result = process_multiple_genomes_single_file(genome_path=genome_path, genes_path=args.genes_path,
                                                          model_name=args.model_name, output_file=str(output_file))
            print("\n✓ GENOME MINIMIZATION COMPLETED!")
            print(f"- Single file generated: {output_file}")
        else:
            print(f"Generating multiple files in: {output_dir}")
            result = process_multiple_genomes_multiple_files(genome_path=genome_path, genes_path=args.genes_path,
                                                             model_name=args.model_name, output_dir=str(output_dir))
            print("\n✓ GENOME MINIMIZATION COMPLETED!")
        print(f"- Processed: {result['genome_count']} genomes")
        print(f"- Average percentage reduction: {result['average_reduction_pct']:.1f}%")
        print(f"- Average genome length: {result['average_length_bp']:,.1f} bp")
        return result
    except Exception as e:
        print(f"✗ Error during genome minimization: {e}")
        traceback.print_exc()
        return None


def main(argv=None):
    args = parse_arguments(argv)
    if args.grad_exchange:
        os.environ["GM2_GRAD_EXCHANGE"] = args.grad_exchange  # read by the trainer's gradient exchange
    if args.sync_bn:
        os.environ["GM2_SYNC_BN"] = "1"  # read by VAETrainer
    dist = None
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        # torchrun: one process per GPU; bind the device and join the process group before any
        # other GPU work (strain-row data parallelism)
        if args.mode not in ("training", "sample"):
            if int(os.environ.get("RANK", "0")) != 0:
                return 0
            print(f"--mode {args.mode} does not shard; running it on rank 0 only")
        else:
            from gm2.ddp import init_from_env
            dist = init_from_env()
    try:
        return _main(args)
    finally:
        if dist is not None:
            dist.destroy_process_group()


def _main(args):
    print(f"\nRunning in {args.mode} mode (MI355X / gfx950 build)")
    if args.mode not in IMPLEMENTED:
        print(f"✗ --mode {args.mode} is outside the MI355X hot path of this build (SURVEY.md §2); "
              "use the reference for it")
        return 2
    if args.mode not in ("convert-samples", "minimizer") and not check_data_availability(args.project_root):
        print("\n✗ Cannot proceed without required data files")
        return 1
    try:
        if args.mode == "sample":
            return 0 if run_sampling(args) else 1
        if args.mode == "convert-samples":
            return 0 if run_binary_converter(args) else 1
        if args.mode == "minimizer":
            if run_genome_minimizer(args) is None:
                return 1
            print("\n" + "=" * 80 + "\nPROCESS COMPLETED!\n" + "=" * 80)
            if args.single_file or args.output_file:
                print("- Check for the generated FASTA file\n")
            else:
                print(f"- Check the {args.output_dir}/ directory for minimized genomes\n")
            return 0
        results = run_single_experiment(args)
        if results is None:
            return 1
    except KeyboardInterrupt:
        print("\n\n✗ Process interrupted by user")
        return 1
    except Exception as e:  # main.py:686-692
        print(f"\n✗ Unexpected error: {e}")
        traceback.print_exc()
        return 1
    print("\n" + "=" * 80 + "\nPROCESS COMPLETED!\n" + "=" * 80)
    return 0


if __name__ == "__main__":
    sys.exit(main())
