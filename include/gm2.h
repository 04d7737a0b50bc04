/*
 * libgm2 — MI355X (gfx950) native VAE train + sample hot path of genome-minimizer-2.
 *
 * C ABI: plain pointers and sizes only. Every pointer argument is a DEVICE pointer owned by the
 * caller (PyTorch's caching allocator in the Python host), except the `const gm2_dims*` /
 * `gm2_batch*` descriptors, which live in host memory. No call allocates device memory; the
 * scratch comes from a caller-allocated workspace whose size `gm2_workspace_size` reports. Every
 * compute call is asynchronous and stream-ordered on the `stream` it is given (a hipStream_t
 * passed as void*). Return value: 0 on success, <0 on error; `gm2_last_error()` then returns a
 * thread-local message. The Python host (gm2/native.py) turns a non-zero return into a
 * RuntimeError, which main.py maps to exit code 1 as the reference does (main.py:686-692).
 *
 * The reference is pure Python (PyTorch eager), so it has no FFI of its own; each entry point
 * below names the reference call site whose work it replaces (paths relative to
 * /root/reference/src/genome_minimizer_2 unless they start with main.py).
 *
 * Parameter layout: ONE flat fp32 buffer holding the 30 tensors of `model.parameters()` in
 * reference order (model.py:65-91: encoder.0.weight, encoder.0.bias, encoder.1.weight, ...,
 * decoder.9.bias), each row-major exactly as in the state_dict. `gm2_param_offsets` gives the
 * offsets. Gradients, Adam exp_avg / exp_avg_sq use the same layout. BatchNorm running
 * statistics: ONE flat fp32 buffer [6][2][H] = (running_mean, running_var) for encoder.1,
 * encoder.4, encoder.7, decoder.1, decoder.4, decoder.7; num_batches_tracked stays on the host.
 */
#ifndef GM2_H
#define GM2_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GM2_ABI_VERSION 6
#define GM2_NUM_PARAMS 30 /* tensors in model.parameters() */
#define GM2_NUM_SCALARS 16

/* arithmetic of the GEMMs: GM2_F32 = exact fp32 MFMA (parity / sampling), GM2_BF16 = bf16 MFMA
 * with fp32 accumulation, fp32 master weights and fp32 BatchNorm / loss / optimizer math */
enum { GM2_F32 = 0, GM2_BF16 = 1 };

/* model + call geometry. G = genes (input_dim), H = hidden_dim (multiple of 128),
 * L = latent_dim (divides 256), batch_max = the largest row count any call will pass. */
typedef struct gm2_dims {
  int64_t G, H, L;
  int64_t batch_max;
} gm2_dims;

/* one batch of strain rows. `data` is the resident u8 presence/absence matrix [n_rows][ld_data]
 * (ld_data a multiple of 16 and >= roundup(G,128), zero padded), `rows` the int32 row indices of
 * this batch (NULL = rows 0..n-1), `eps` the N(0,1) draws of model.py:102 as fp32 [n][L]. */
typedef struct gm2_batch {
  const uint8_t* data;
  int64_t ld_data;
  const int32_t* rows;
  int64_t n;
  const float* eps;
  /* optional (gm2_train_fwd_bwd only): the batch the NEXT gm2_train_fwd_bwd on this workspace will
   * be given. Its rows are gathered into the workspace's second input slot on the library's side
   * stream while this call's input-layer weight-gradient GEMM runs; the next call, given a batch
   * with the same data / ld_data / rows / n, then skips its own gather. The memory `next` points at
   * (data, rows) must stay unchanged until that call; eps is not read. Any other call that gathers
   * rows (eval, encode, forward, recon counts) first waits for and discards a pending stage. */
  const struct gm2_batch* next;
  /* optional (ABI 4): the resident matrix as GEMM operands, built once by gm2_resident_build from
   * the same data. When set (resident_prec = the workspace precision) gm2_train_fwd_bwd reads the
   * batch's rows IN PLACE: the input-layer GEMMs take rows resident[rows[i]] of the [S + 1][ld]
   * matrix and the loss epilogue the matching target-bit rows, so no rows are gathered (next is
   * then not staged). Used when the plans allow it (bf16 workspace, 256x256 tiles, rows padded to a
   * multiple of 256, ld_resident >= the workspace's padded G); otherwise the call gathers from
   * data as before. Other calls always gather. Zero-initialised (NULL) = not used. */
  const void* resident;          /* T [resident_rows + 1 (zero row) ...][ld_resident], pad columns zero */
  int64_t ld_resident;           /* elements, multiple of 64 */
  const uint32_t* resident_bits; /* [...][ld_resident_bits] packed target bits (bit g % 32 of word g / 32) */
  int64_t ld_resident_bits;      /* 32-bit words, multiple of 4 */
  int64_t resident_rows;         /* S: the data rows; row S of both arrays is all zero */
  int resident_prec;             /* GM2_F32 / GM2_BF16: the element type of `resident` */
} gm2_batch;

/* device scalar block (fp32[GM2_NUM_SCALARS]) read by the kernels, written by the host per step
 * so a captured graph can replay: */
enum {
  GM2_S_BETA = 0,          /* KL weight (loss_components.py:76-88)                         */
  GM2_S_WGAMMA = 1,        /* weight * gamma of GeneAbundanceLoss (0 = absent)              */
  GM2_S_LAMBDA = 2,        /* lambda_l1 (0 = absent)                                        */
  GM2_S_NEG_STEP = 3,      /* -lr / (1 - beta1^t)                                           */
  GM2_S_BC2_SQRT = 4,      /* sqrt(1 - beta2^t)                                             */
  GM2_S_MAX_NORM = 5,      /* clip_grad_norm_ max_norm (<= 0: no clipping)                  */
  GM2_S_ONE_MINUS_B1 = 6,
  GM2_S_BETA2 = 7,
  GM2_S_ONE_MINUS_B2 = 8,
  GM2_S_ADAM_EPS = 9,
  GM2_S_NORM_AHEAD = 10    /* != 0: `grads` reaches gm2_grad_norm exactly as the last
                              gm2_train_fwd_bwd on this workspace wrote it (one process, no
                              exchange or edit in between); the clip statistics of the two big
                              weight gradients are then taken from that call's GEMM epilogues
                              instead of a second pass over 2*H*G floats. 0 = always re-read. */
};

/* loss record (fp64[GM2_LOSS_SLOTS], device) filled per call:
 *   [0] sum of BCE elements           (ReconstructionLoss, loss_components.py:49-50)
 *   [1] sum of reconstructed p        (GeneAbundanceLoss before w*gamma; p >= 0 so |.| = id)
 *   [2] sum(1 + lv - mu^2 - exp(lv))  (KLDivergenceLoss before -0.5*beta)
 *   [3] sum |theta| over all params   (l1_regularization before lambda; gm2_grad_norm; only
 *                                      when lambda != 0, else 0 — the reference returns 0 then)
 *   [4] total gradient L2 norm after L1 (clip_grad_norm_ total_norm; gm2_grad_norm)       */
#define GM2_LOSS_SLOTS 8

const char* gm2_last_error(void);
int gm2_abi_version(void);

/* sizes / layout queries (host only) */
int gm2_param_count(const gm2_dims* d, int64_t* n_params);
int gm2_param_offsets(const gm2_dims* d, int64_t* offsets /* [GM2_NUM_PARAMS + 1] */);
int gm2_workspace_size(const gm2_dims* d, int precision, size_t* bytes);

/* Initialise a workspace (zero it, lay out GEMM shadows and pads). Call once after allocation.
 * The library keeps a little host-side state per workspace, keyed by its address: its tuning
 * options (copied from the process defaults here), its side stream, its gradient-bucket events and
 * its staged input slot. Nothing is shared between workspaces, so two models (or a training and a
 * sampling workspace) can be used in one process; one workspace is used from one host thread at a
 * time. gm2_workspace_release drops that state (call it before freeing the device memory). A
 * still-QUEUED output-layer Adam update (GM2_OPT_DEFER_OUTPUT_ADAM) is discarded, not launched
 * (release may run after the parameter buffers it would write were freed): call gm2_workspace_join
 * first to keep it. Returns 1 (with gm2_last_error saying so) when an update was discarded, 0 when
 * nothing was pending; the state is released either way. */
int gm2_workspace_init(const gm2_dims* d, int precision, void* ws, size_t ws_bytes, void* stream);
int gm2_workspace_release(void* ws);

/* Re-derive the padded GEMM copies of the Linear weights from `params` (after init,
 * load_state_dict, or any host-side edit). gm2_adam_step keeps them current itself. */
int gm2_sync_shadows(const gm2_dims* d, int precision, const float* params, void* ws, void* stream);

/* Resident-matrix operands (gm2_batch.resident), built once from the 0/1 u8 rows data [S][ld_data]:
 * gm2_resident_layout gives the element pitch ld (roundup(G, 256)), the bit-row pitch ld_bits
 * (ld / 32 words), the row count to allocate (roundup(S + 1, 64): row S and beyond are zero) and the
 * byte sizes of the two arrays; gm2_resident_build fills them (T = float or bf16 by prec). */
int gm2_resident_layout(int64_t S, int64_t G, int prec, int64_t* ld, int64_t* ld_bits, int64_t* rows_alloc,
                        size_t* bytes, size_t* bits_bytes);
int gm2_resident_build(const uint8_t* data, int64_t ld_data, int64_t S, int64_t G, int prec, void* out,
                       uint32_t* bits, void* stream);

/* Training forward + backward of one batch (replaces trainer.py:110-118: model(data),
 * compute_total_loss, total_loss.backward()). Overwrites `grads` with the data-term gradient
 * (reconstruction + beta*KL + abundance; the L1 term is added by gm2_grad_norm/gm2_adam_step),
 * updates BN running stats (train-mode BatchNorm, model.py:67-86), writes loss slots [0..2]. */
int gm2_train_fwd_bwd(const gm2_dims* d, int precision, const gm2_batch* batch, const float* params,
                      float* grads, float* bn_running, const float* scalars, double* loss, void* ws,
                      void* stream);

/* Data-parallel gradient exchange. The flat gradient buffer is cut into
 * GM2_GRAD_BUCKETS contiguous ranges in the order gm2_train_fwd_bwd finalises them:
 *   0 = decoder.9.{weight,bias}, 1 = encoder.0.bias .. decoder.7.bias,
 *   2..5 = encoder.0.weight rows in four contiguous quarters (of H rows each rounded to whole
 *          rows; with GM2_OPT_INPUT_CHUNKS = 4 each quarter is final after its own launch, so the
 *          exchange of the first quarters runs under the GEMM of the later ones).
 * gm2_grad_bucket_bounds writes [lo, hi) element offsets per bucket (lo_hi[2*GM2_GRAD_BUCKETS]).
 * gm2_wait_grad_bucket makes `stream` wait (device-side, no host sync) until that bucket of the
 * most recent gm2_train_fwd_bwd / gm2_backward_outputs on workspace `ws` is written, so a caller
 * can start the all-reduce of bucket b on a communication stream while the rest of that backward
 * still runs. Call it after the backward it refers to and before the next one on `ws`. */
#define GM2_GRAD_BUCKETS 6
int gm2_grad_bucket_bounds(const gm2_dims* d, int64_t* lo_hi);
int gm2_wait_grad_bucket(void* ws, int bucket, void* stream);

/* The bf16 exchange of the big weight-gradient buckets (gm2/ddp.py bf16_exchange_sum; the reference
 * is single-device): every rank rounds its bucket to bf16 once (pack), sends chunk j to
 * rank j (all-to-all, the caller's collective), rank j sums the world's chunks in fp32 IN RANK ORDER
 * and rounds the sum to bf16 once (ranksum), an all-gather hands every rank every chunk, and unpack
 * widens it back into the fp32 gradient. Device pointers, stream-ordered, no allocation.
 *   gm2_exchange_pack     out[i] = bf16_rne(x[i]) for i < n, 0 for n <= i < n_pad (out 16-B aligned)
 *   gm2_exchange_ranksum  out[i] = bf16_rne((((float)parts[0][i] + parts[1][i]) + ...) + parts[world-1][i]),
 *                         parts = world chunks of `chunk` elements back to back (chunk % 8 == 0)
 *   gm2_exchange_unpack   x[i] = (float)in[i], i < n */
int gm2_exchange_pack(const float* x, int64_t n, uint16_t* out, int64_t n_pad, void* stream);
int gm2_exchange_ranksum(const uint16_t* parts, int world, int64_t chunk, uint16_t* out, void* stream);
int gm2_exchange_unpack(const uint16_t* in, int64_t n, float* x, void* stream);

/* L1 term + clip_grad_norm_ statistics (trainer.py:119; loss_components.py:167-184): computes
 * ||g + lambda*sign(theta)||_2 (loss slot [4]), sum|theta| (slot [3]) and the clip coefficient
 * min(1, max_norm/(norm+1e-6)) kept in the workspace for gm2_adam_step. */
int gm2_grad_norm(const gm2_dims* d, int precision, const float* params, const float* grads,
                  const float* scalars, double* loss, void* ws, void* stream);

/* torch.optim.Adam step (trainer.py:120; lr from StepLR, experiments.py:260-265) on
 * (grads + lambda*sign(theta)) * clip, then refreshes the GEMM shadows. */
int gm2_adam_step(const gm2_dims* d, int precision, float* params, const float* grads, float* exp_avg,
                  float* exp_avg_sq, const float* scalars, void* ws, void* stream);

/* Validation forward (trainer.py:139-149): eval-mode BatchNorm (running stats), reparam with the
 * given eps, loss slots [0..2]; nothing else is written. */
int gm2_eval_forward(const gm2_dims* d, int precision, const gm2_batch* batch, const float* params,
                     const float* bn_running, const float* scalars, double* loss, void* ws, void* stream);

/* Sampling decode (extras.py:192-203, main.py:351-370): z fp32 [n][L] -> eval-mode decoder (hidden
 * layers in exact fp32; the output layer gated per tile between bf16x3 and exact fp32 with an fp64
 * recompute of the certified band, GM2_OPT_SAMPLE_SPLIT) -> mask u8 [n][ld_mask] =
 * (sigmoid(logit) > 0.5), optionally probs fp32 [n][ld_probs] (NULL to skip; a probs request runs
 * the whole output layer in exact fp32). n <= batch_max. */
int gm2_decode_mask(const gm2_dims* d, const float* params, const float* bn_running, const float* z,
                    int64_t n, uint8_t* mask, int64_t ld_mask, float* probs, int64_t ld_probs, void* ws,
                    void* stream);

/* Packed sampled masks: numpy packbits(bitorder='little') rows, bit (g & 7) of byte g / 8 = gene g,
 * row pitch ld_bits >= gm2_packed_row_bytes(G) (a multiple of 16), bits beyond G zero. 8x less HBM
 * and PCIe than the u8 mask; what --mode sample keeps on the device for the mask consumers. */
int64_t gm2_packed_row_bytes(int64_t G);

/* gm2_decode_mask with a packed output: bits [n][ld_bits] (+ optional probs). */
int gm2_decode_bits(const gm2_dims* d, const float* params, const float* bn_running, const float* z, int64_t n,
                    uint8_t* bits, int64_t ld_bits, float* probs, int64_t ld_probs, void* ws, void* stream);

/* count_essential_genes (extras.py:49-87) on packed masks: counts[i] = number of groups g (essential
 * genes) with ANY set position in positions[group_offsets[g] .. group_offsets[g+1]) (all < G). */
int gm2_mask_count_groups(const uint8_t* bits, int64_t n, int64_t ld_bits, const int32_t* group_offsets,
                          int64_t n_groups, const int32_t* positions, int32_t* counts, void* stream);

/* masks_to_gene_lists (binary_converter.py:19-76) as a CSR of gene column indices: offsets[n+1]
 * (int64, exclusive scan of the row popcounts of bits AND keep_bits), then the ascending set
 * columns of every row at indices[offsets[i] ..]. keep_bits (one packed row, NULL = all) drops
 * duplicate gene names (binary_converter.py:29-36 keeps the first occurrence). */
int gm2_mask_row_offsets(const uint8_t* bits, int64_t n, int64_t ld_bits, const uint8_t* keep_bits, int64_t* offsets,
                         void* stream);
int gm2_mask_compact(const uint8_t* bits, int64_t n, int64_t ld_bits, const uint8_t* keep_bits, const int64_t* offsets,
                     int32_t* indices, void* stream);

/* calculate_reconstruction_metrics (training/evaluation/metrics.py:19-64) without materialising the
 * reconstruction: eval-mode model(x) of `batch` (eps given: the reference samples z there too), then
 * per strain counts[i] = (TP, FP, FN) of (recon > threshold) against the strain's genes. */
int gm2_recon_counts(const gm2_dims* d, int precision, const gm2_batch* batch, const float* params,
                     const float* bn_running, float threshold, int32_t* counts, void* ws, void* stream);

/* Encoder of VAE.encode (model.py:95-98), eval-mode BatchNorm, on `batch` (eps unused):
 * mu and logvar fp32 [n][L] (either may be NULL). Used by get_latent_variables (extras.py:205-228). */
int gm2_encode(const gm2_dims* d, int precision, const gm2_batch* batch, const float* params,
               const float* bn_running, float* mu, float* logvar, void* ws, void* stream);

/* VAE.forward (model.py:109-113) as `model(x)`: encoder (BatchNorm in train mode — batch
 * statistics + running-stat update — when `train`, else running stats), reparameterisation with
 * the given batch->eps, decoder, probs fp32 [n][ld_probs] = sigmoid(logits); mu / logvar fp32 [n][L]
 * (either may be NULL). The workspace keeps the activations for gm2_backward_outputs. */
int gm2_forward(const gm2_dims* d, int precision, const gm2_batch* batch, const float* params, float* bn_running,
                int train, float* probs, int64_t ld_probs, float* mu, float* logvar, void* ws, void* stream);

/* Backward of the most recent gm2_forward on this workspace (same batch, same `train` mode) given
 * upstream gradients dL/dprobs [n][ld_probs], dL/dmu and dL/dlogvar [n][L] (either may be NULL) —
 * what torch autograd hands back to VAE.forward when a custom LossComponent is trained
 * (trainer.py:349-352 with_custom_loss). Overwrites `grads` (flat, parameter order) with dL/dtheta
 * through the whole VAE (train = 0: eval-mode BatchNorm, an affine map). */
int gm2_backward_outputs(const gm2_dims* d, int precision, const gm2_batch* batch, const float* params, int train,
                         const float* probs, int64_t ld_probs, const float* dprobs, const float* dmu,
                         const float* dlogvar, float* grads, void* ws, void* stream);

/* VAE.reparameterization (model.py:100-104) with the noise given: z = mu + exp(0.5*logvar)*eps over
 * n elements; with dz != NULL also (or only, z = NULL) its backward dmu = dz,
 * dlogvar = 0.5*dz*eps*exp(0.5*logvar). */
int gm2_reparameterize(int64_t n, const float* mu, const float* logvar, const float* eps, float* z,
                       const float* dz, float* dmu, float* dlogvar, void* stream);

/* Raw GEMM primitive, exposed for kernel-level tests: C[M][ldc] (fp32) = sum_k P(m,k) Q(n,k).
 * p_kmajor / q_kmajor = 1: the operand is stored [rows][ld] with K contiguous (P(m,k) = P[m*ld+k]);
 * 0: stored [K][ld] with M (N) contiguous (P(m,k) = P[k*ld+m]). Elements of `precision` type;
 * the M (N) extent is padded to a multiple of 128 in the allocation, K % 64 == 0, pads zero.
 * (P MN-major with Q K-major is not instantiated.) splits 0/1: one pass straight into C; > 1: that
 * many split-K slices; < 0: the hot path's own tile / split plan (at most 32 slices). Split runs
 * need slab_ws (fp32, splits * M * ldc elements) and sum the slices into C. */
int gm2_gemm(int precision, int p_kmajor, int q_kmajor, const void* P, int64_t ldp, const void* Q,
             int64_t ldq, float* C, int64_t ldc, int64_t M, int64_t N, int64_t K, int splits,
             float* slab_ws, void* stream);

/* Live kernel timing for the benchmark's roofline figure: between gm2_timing_begin(classes) and
 * gm2_timing_end, every launch of a selected kernel class is bracketed by a hipEvent pair on its
 * own stream; gm2_timing_end synchronises those events and returns their summed duration and the
 * launch count. Classes: GM2_KC_RECON_LOSS (decoder output layer GEMM + fused BCE / dlogits
 * epilogue), GM2_KC_GEMM_STORE (every other GEMM), GM2_KC_MASK (sampling output layer GEMM). */
/* Tuning switches (no effect on results' semantics; every value is parity-tested). Each workspace
 * has its own set: gm2_workspace_set_option / gm2_workspace_get_option edit / read it and act on
 * the calls that use that workspace. gm2_set_option / gm2_get_option edit / read the PROCESS
 * DEFAULTS: the set a workspace receives at gm2_workspace_init, and the one gm2_gemm (no
 * workspace) runs with.
 *   GM2_OPT_GEMM_PP     1 = ping-pong (4-phase, staggered wave groups) main loop for the 256x256
 *                       bf16 GEMM tiles (default), 0 = two-stage loop. Process default from env
 *                       GM2_GEMM_PP (0 disables).
 *   GM2_OPT_SIDE_STREAM 1 = weight-gradient GEMMs on the workspace's forked side stream (default),
 *                       0 = all on the caller's stream. Process default from env GM2_SIDE_STREAM.
 *   GM2_OPT_RECON_TILE  output-layer loss GEMM tile: 0 = plan (default), 128 or 256 = force.
 *   GM2_OPT_SMALL_SPLIT split-K factor (1..8) of the chip-filling short-K 128-tile GEMMs (the
 *                       hidden layers).
 *   GM2_OPT_BN_EPILOGUE 1 = BatchNorm batch statistics (forward) and backward partial sums taken
 *                       in the producing GEMM's store epilogue where the plan allows (default),
 *                       0 = always a separate statistics pass.
 *   GM2_OPT_SMALL_WAVES waves per workgroup (4 or 8) of the 128x128 fp32-store GEMM tiles (the
 *                       hidden-layer GEMMs).
 *   GM2_OPT_GRID_CAP    bit 1 = the output-layer, bit 2 = the input-layer weight-gradient GEMM,
 *                       bit 4 = the output-layer loss GEMM runs on a capped grid (workgroups loop over tiles; same rounds, fewer CUs)
 *                       so the work beside it keeps CUs (default 3: both weight gradients); 0 = one
 *                       workgroup per tile.
 *   GM2_OPT_INPUT_CHUNKS 1 (default) or 4: launches of the input-layer weight-gradient GEMM, one
 *                       per gradient bucket 2..5 (when H/4 is a multiple of 256; else 1). Same
 *                       results bit for bit; 4 lets a data-parallel exchange start early.
 *   GM2_OPT_SYNC_BN     (workspace option; changes the model's semantics on purpose) 1 = SyncBN for
 *                       data-parallel training: train-mode BatchNorm normalises with the statistics
 *                       of the GLOBAL batch (every rank's rows), as the single-device reference does
 *                       (model.py:67-86), instead of each rank's own rows. Needs a collective
 *                       (gm2_workspace_set_collective): per training call the library all-reduces
 *                       (SUM, fp64) 6 forward [sum y | sum y^2 | rows] and 6 backward
 *                       [sum do | sum (y-mean) do | rows] vectors of 2H+2 doubles, in a fixed order
 *                       (forward layers encoder.1 .. decoder.7, then backward decoder.7 .. encoder.1).
 *                       A rank with no rows in a global batch calls gm2_train_fwd_bwd with n = 0: it
 *                       takes part in the 12 all-reduces with zeros, writes zero gradients and loss
 *                       slots, and applies the same running-statistics update. Default 0.
 *   GM2_OPT_DEFER_OUTPUT_ADAM (workspace option) n >= 1 = gm2_adam_step updates every tensor but the
 *                       output layer (decoder.9.weight / .bias, half the optimizer's bytes at v0)
 *                       on the caller's stream and returns with the output layer's update QUEUED
 *                       (its scalar block copied into the workspace): the next training call
 *                       launches it on the workspace's side stream right after its input-layer
 *                       GEMM, on n workgroups per CU (1..16) beside the hidden layers, and waits
 *                       for it before the output layer. 0 = not deferred (default).
 *                       Results are bit-identical. Until then the output layer's parameters /
 *                       moments are not updated: read them only after gm2_workspace_join (every
 *                       other libgm2 call on the workspace joins first, which launches a queued
 *                       update on its stream), and keep the buffers passed to gm2_adam_step alive.
 *   GM2_OPT_GRAD_BUCKETS (workspace option) 1 = gm2_train_fwd_bwd records the gradient-bucket
 *                       events gm2_wait_grad_bucket waits on (default); 0 = it records none (each
 *                       is a system-scope release on the stream: ~7 us of idle GPU apiece), and
 *                       gm2_wait_grad_bucket fails. For a single process that exchanges nothing.
 *   GM2_OPT_SAMPLE_SPLIT 1 (default) = gm2_decode_mask / gm2_decode_bits without probs run the output
 *                       layer gated per 256 x 256 tile: as one bf16 GEMM over 2H (the fp32
 *                       activations and weights split into bf16 hi + lo, summing hi.hi + hi.lo +
 *                       lo.hi per K-tile) where 4.62e-5 x the tile's largest ||a_r||_2 x its largest
 *                       ||w_g||_2 is at most 1e-3, in exact fp32 elsewhere; logits in the certified
 *                       band around the threshold are then recomputed in fp64 (GM2_STAT_BAND_*), so
 *                       a mask bit differs from the correctly rounded logit's only within the
 *                       reference's own fp32 rounding band. 0 = always the exact-fp32 output layer
 *                       without band recompute (as do probs requests).
 *   GM2_OPT_SAMPLE_SINGLE 1 (default) = a third tier of that gate: tiles where 7.83e-3 x the tile's
 *                       largest ||a_r||_2 x its largest ||w_g||_2 is at most 0.25 run ONE bf16 GEMM
 *                       over the rounded operands (a third of the split's MFMA work) with a
 *                       correspondingly wider certified band, recomputed in fp64 the same way;
 *                       0 = split or exact only.
 *   GM2_OPT_SAMPLE_BAND_CAP (ABI 6) entries per shard of the certified band's list per decode call
 *                       (1..65536, default 65536; 64 shards). Entries past a shard's capacity are
 *                       not dropped: their 256 x 256 output block (genome rows x genes) is recomputed
 *                       whole in fp64 after the band recompute (GM2_STAT_OVERFLOW_TILES), so the
 *                       masks do not depend on this value; smaller values exercise that path.
 *   GM2_OPT_SAMPLE_SINGLE_BOUND (ABI 6) the single tier's gate x 1000 (default 250 = 0.25, 1..1e6):
 *                       larger values send more tiles to the single tier (a wider band; a tile
 *                       whose band overflows its slots re-runs as bf16x3). Cost only, never the masks. */
enum {
  GM2_OPT_GEMM_PP = 1,
  GM2_OPT_SIDE_STREAM = 2,
  GM2_OPT_RECON_TILE = 3,
  GM2_OPT_SMALL_SPLIT = 4,
  GM2_OPT_BN_EPILOGUE = 5,
  GM2_OPT_SMALL_WAVES = 6,
  GM2_OPT_INPUT_CHUNKS = 7,
  GM2_OPT_GRID_CAP = 9,
  GM2_OPT_SYNC_BN = 10,
  GM2_OPT_DEFER_OUTPUT_ADAM = 11,
  GM2_OPT_GRAD_BUCKETS = 15,
  GM2_OPT_SAMPLE_SPLIT = 18,
  GM2_OPT_SAMPLE_SINGLE = 20,
  GM2_OPT_SAMPLE_BAND_CAP = 21,
  GM2_OPT_SAMPLE_SINGLE_BOUND = 22
};
int gm2_set_option(int key, int value);
int gm2_get_option(int key, int* value);
int gm2_workspace_set_option(void* ws, int key, int value);
int gm2_workspace_get_option(void* ws, int key, int* value);
/* Make `stream` wait for work the workspace left running on its side stream (a deferred output-
 * layer Adam update, GM2_OPT_DEFER_OUTPUT_ADAM); no-op when nothing is pending. */
int gm2_workspace_join(void* ws, void* stream);
/* Counters of a workspace's sampling decodes (gm2_decode_mask / gm2_decode_bits), cumulative since
 * gm2_workspace_init; reading one waits for the device.
 *   GM2_STAT_SPLIT_DECODES  decodes whose output layer ran at least one tile as bf16x3 or single
 *                           bf16 (GM2_OPT_SAMPLE_SPLIT, GM2_OPT_SAMPLE_SINGLE)
 *   GM2_STAT_EXACT_DECODES  decodes with no such tile (the gate's verdict, a probs request,
 *                           GM2_OPT_SAMPLE_SPLIT off, or the split path's preconditions)
 *   GM2_STAT_SPLIT_TILES / GM2_STAT_EXACT_TILES  output-layer tiles (256 x 256 split, 128 x 128 exact)
 *                           each kernel of the gated decode ran
 *   GM2_STAT_BAND_ELEMENTS  logits the gated decode flagged in the certified band |logit - T| <=
 *                           coef * ||a_r||_2 ||w_g||_2 (evaluated with the largest
 *                           of 4 neighbouring rows' norms, so a small superset) and recomputed in fp64
 *   GM2_STAT_BAND_FLIPS     mask bits that recompute changed
 *   GM2_STAT_BAND_OVERFLOW  band elements beyond a call's list capacity (256 slots per split
 *                           tile, then 64 shards x GM2_OPT_SAMPLE_BAND_CAP); each one's 256 x 256
 *                           block is recomputed whole in fp64 (ABI 6: no bit is left as computed)
 *   GM2_STAT_SINGLE_TILES   output-layer tiles (256 x 256) the single-product kernel ran
 *   GM2_STAT_OVERFLOW_TILES 256 x 256 blocks recomputed whole in fp64 after a list overflow */
enum {
  GM2_STAT_SPLIT_DECODES = 1,
  GM2_STAT_EXACT_DECODES = 2,
  GM2_STAT_SPLIT_TILES = 3,
  GM2_STAT_EXACT_TILES = 4,
  GM2_STAT_BAND_ELEMENTS = 5,
  GM2_STAT_BAND_FLIPS = 6,
  GM2_STAT_BAND_OVERFLOW = 7,
  GM2_STAT_SINGLE_TILES = 8,
  GM2_STAT_OVERFLOW_TILES = 9
};
int gm2_workspace_stat(void* ws, int key, int64_t* value);

/* The all-reduce SyncBN needs (GM2_OPT_SYNC_BN), supplied by the caller: SUM `count` doubles at the
 * DEVICE pointer `buf` (inside the workspace) across every rank, in place, ordered on `stream` (the
 * stream of the libgm2 call in progress: work enqueued on it before the call must be done before
 * the reduction reads `buf`, and work enqueued after the callback returns must see the result).
 * Returns 0 on success. Called from inside gm2_train_fwd_bwd on the calling thread. The Python host
 * binds torch.distributed.all_reduce (RCCL) here (gm2/ddp.py). */
typedef int (*gm2_allreduce_fn)(double* buf, int64_t count, void* stream, void* user);
int gm2_workspace_set_collective(void* ws, gm2_allreduce_fn fn, void* user);

enum { GM2_KC_RECON_LOSS = 1, GM2_KC_GEMM_STORE = 2, GM2_KC_MASK = 4, GM2_KC_ADAM = 8 };
int gm2_timing_begin(int kernel_classes);
int gm2_timing_end(double* total_ms, int64_t* launches);
/* (ABI 6) after gm2_timing_end: the summed duration and launch count of ONE of the classes that were
 * timed together (GM2_KC_ADAM: the fused L1 + clip + Adam passes, the deferred one included) */
int gm2_timing_class(int kernel_class, double* total_ms, int64_t* launches);

#ifdef __cplusplus
}
#endif
#endif /* GM2_H */
