"""Presets + experiment runner — mirror of src/genome_minimizer_2/utils/experiments.py.

get_v{0..3}_config (:42-114) verbatim; IntegratedExperimentRunner keeps the hot-path stages of
run_complete_experiment (:424-444): prep_data (:195-223), create_dataloaders (:225-252),
setup_model_and_training (:254-270), display_config (:147-193) and train_model + the state_dict
save (:272-329). Post-training plots / metrics / PCA (:331-422) are out of scope (SURVEY.md §2
rows 10-11) and are skipped with a log line.
"""
from __future__ import annotations

import logging
import os
from datetime import datetime
from pathlib import Path

import torch

from . import native
from .custom_config import ExperimentConfig
from .data import ResidentMatrix, StrainLoader, load_and_validate_data, split_indices
from .ddp import broadcast_model, get_dist, rank_world, shared_seed
from .model import VAE
from .trainer import Adam, StepLR, v0, v1, v2, v3

logging.basicConfig(level=logging.INFO, format="%(asctime)s - %(levelname)s - %(message)s")
logger = logging.getLogger(__name__)


def get_v0_config() -> ExperimentConfig:
    return ExperimentConfig(hidden_dim=1024, latent_dim=64, n_epochs=10000, min_beta=0.1, max_beta=1.0,
                            lambda_l1=0.0, trainer_version="v0", experiment_name="v0_model")


def get_v1_config() -> ExperimentConfig:
    return ExperimentConfig(hidden_dim=512, latent_dim=32, n_epochs=10000, min_beta=0.1, max_beta=1.0,
                            gamma_start=1.0, gamma_end=0.1, lambda_l1=0.01, trainer_version="v1",
                            experiment_name="v1_model")


def get_v2_config() -> ExperimentConfig:
    return ExperimentConfig(hidden_dim=512, latent_dim=32, n_epochs=10000, min_beta=0.0, max_beta=1.0,
                            gamma_start=1.0, gamma_end=0.1, lambda_l1=0.01, trainer_version="v2",
                            experiment_name="v2_model")


def get_v3_config() -> ExperimentConfig:
    return ExperimentConfig(hidden_dim=512, latent_dim=32, n_epochs=10000, min_beta=0.1, max_beta=1.0,
                            gamma_start=2.0, gamma_end=0.1, weight=1.0, lambda_l1=0.01, trainer_version="v3",
                            experiment_name="v3_model")


PRESETS = {"v0": get_v0_config, "v1": get_v1_config, "v2": get_v2_config, "v3": get_v3_config}


def run_preset(config, model, optimizer, scheduler, train_loader, val_loader, folder="./", **kw):
    """Dispatch to v0..v3 with the argument lists of experiments.py:280-311."""
    c = config
    if c.trainer_version == "v0":
        return v0(model, folder, optimizer, scheduler, c.n_epochs, train_loader, val_loader, c.min_beta, c.max_beta,
                  c.max_norm, **kw)
    if c.trainer_version == "v1":
        return v1(model, folder, optimizer, scheduler, c.n_epochs, train_loader, val_loader, c.min_beta, c.max_beta,
                  c.gamma_start, c.gamma_end, c.max_norm, c.lambda_l1, **kw)
    if c.trainer_version == "v2":
        return v2(model, folder, optimizer, scheduler, c.n_epochs, train_loader, val_loader, c.min_beta, c.max_beta,
                  c.gamma_start, c.gamma_end, c.max_norm, c.lambda_l1, **kw)
    if c.trainer_version == "v3":
        return v3(model, folder, optimizer, scheduler, c.n_epochs, train_loader, val_loader, c.min_beta, c.max_beta,
                  c.gamma_start, c.gamma_end, c.weight, c.max_norm, c.lambda_l1, **kw)
    raise ValueError(f"Unknown trainer version: {c.trainer_version}")


class IntegratedExperimentRunner:
    def __init__(self, config: ExperimentConfig, project_root=None, precision=native.GM2_BF16, dataset_csv=None,
                 phylogroups_csv=None):
        self.config = config
        self.project_root = project_root or os.environ.get("GM2_PROJECT_ROOT", os.getcwd())
        self.precision = precision
        self.dataset_csv = dataset_csv or os.path.join(self.project_root, "data", "F4_complete_presence_absence.csv")
        self.phylogroups_csv = phylogroups_csv or os.path.join(self.project_root, "data",
                                                               "accessionID_phylogroup_BD.csv")
        self.logger = logging.getLogger(f"{__name__}.{config.experiment_name}")
        self.figure_dir = os.path.join(self.project_root, "models", config.experiment_name, "figures")
        self.model_dir = os.path.join(self.project_root, "models", "trained_models", config.experiment_name)
        os.makedirs(self.figure_dir, exist_ok=True)
        os.makedirs(self.model_dir, exist_ok=True)
        self.results = {}
        self.device = torch.device("cuda", torch.cuda.current_device())
        self.logger.info(f"Using device: {self.device}")

    def display_config(self):
        if rank_world()[0] != 0:
            return
        lines = ["=" * 80, "EXPERIMENT CONFIGURATION", "=" * 80,
                 f"Generated on: {datetime.now().strftime('%Y-%m-%d %H:%M:%S')}", ""]
        cats = {"Model Parameters": ["hidden_dim", "latent_dim"],
                "Training Parameters": ["n_epochs", "batch_size", "learning_rate", "max_norm", "lambda_l1"],
                "Loss Scheduling": ["min_beta", "max_beta", "gamma_start", "gamma_end", "weight"],
                "Trainer": ["trainer_version"], "Scheduler": ["scheduler_step_size", "scheduler_gamma"],
                "Data Split": ["test_size", "val_ratio", "random_state"],
                "Output": ["experiment_name", "save_model", "generate_plots", "calculate_metrics",
                           "explore_latent_space"]}
        for cat, ps in cats.items():
            lines += [f"{cat}:", "-" * len(cat)]
            lines += [f"  {p:<20}: {getattr(self.config, p)}" for p in ps]
            lines.append("")
        lines.append("=" * 80)
        text = "\n".join(lines)
        print(text)
        Path(self.figure_dir, f"{self.config.experiment_name}_config.txt").write_text(text)

    def prep_data(self):
        dist = get_dist()
        if dist:
            # one host RNG stream on every rank: same loader permutations and eps draws
            torch.manual_seed(shared_seed(dist))
        _, merged, _ = load_and_validate_data(self.dataset_csv, self.phylogroups_csv)
        data = merged.iloc[:, :-1].values
        self.phylogroups = merged["Phylogroup"].values
        self.input_dim = data.shape[1]
        self.create_dataloaders(data, self.phylogroups, self.config.batch_size)

    def create_dataloaders(self, data_array, labels, batch_size):
        tr, va, te = split_indices(len(data_array), self.config.test_size, self.config.val_ratio,
                                   self.config.random_state)
        self.logger.info(f"Data splits - Train: {len(tr)}, Val: {len(va)}, Test: {len(te)}")
        self.matrix = ResidentMatrix(data_array, device=self.device)
        self.train_loader = StrainLoader(self.matrix, tr, batch_size, shuffle=True)
        self.val_loader = StrainLoader(self.matrix, va, batch_size, shuffle=False)
        self.test_loader = StrainLoader(self.matrix, te, batch_size, shuffle=False)
        self.test_phylogroups = labels[te]

    def setup_model_and_training(self):
        c = self.config
        self.model = VAE(self.input_dim, c.hidden_dim, c.latent_dim, device=self.device, precision=self.precision)
        self.optimizer = Adam(self.model, lr=c.learning_rate)
        self.scheduler = StepLR(self.optimizer, step_size=c.scheduler_step_size, gamma=c.scheduler_gamma)
        dist = get_dist()
        if dist:
            broadcast_model(dist, self.model)
        self.logger.info(f"Model parameters - Total: {self.model.n_params:,}, Trainable: {self.model.n_params:,}")

    def train_model(self, **kw):
        c = self.config
        self.logger.info(f"Starting training with {c.trainer_version} configuration...")
        tr, va, ep = run_preset(c, self.model, self.optimizer, self.scheduler, self.train_loader, self.val_loader,
                                self.figure_dir + "/", **kw)
        self.results.update(train_loss_vals=tr, val_loss_vals=va, epochs_trained=ep)
        self.logger.info(f"Training completed after {ep} epochs")
        self.logger.info(f"Final train loss: {tr[-1]:.4f}")
        self.logger.info(f"Final validation loss: {va[-1]:.4f}")
        if c.save_model and rank_world()[0] == 0:
            path = os.path.join(self.model_dir, f"saved_VAE_{c.trainer_version}.pt")
            torch.save(self.model.state_dict(), path)
            self.results["model_path"] = path
            self.logger.info(f"Model saved to {path}")

    def run_complete_experiment(self, **kw):
        self.logger.info(f"** START OF EXPERIMENT: {self.config.experiment_name} **")
        self.prep_data()
        self.setup_model_and_training()
        self.display_config()
        self.train_model(**kw)
        self.logger.info("Post-training plots / F1 metrics / latent PCA are outside the MI355X hot path; skipped")
        self.logger.info(f"** EXPERIMENT {self.config.experiment_name} COMPLETED SUCCESSFULLY **")
        return self.results
