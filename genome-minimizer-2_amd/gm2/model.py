"""VAE — MI355X mirror of the reference model (src/genome_minimizer_2/training/model.py:13-120).

Same constructor, same state_dict keys / shapes / dtypes, same init RNG replay, same
encode / reparameterization / decode / forward contract. The difference is the storage: all 30
parameter tensors live in ONE flat fp32 device buffer (reference order, model.py:65-91) and all
6 BatchNorm running statistics in one [6][2][H] buffer, which is what libgm2's kernels consume.
Every compute method runs through libgm2.so; there is no PyTorch-op fallback.
"""
from __future__ import annotations

import math
from collections import OrderedDict

import torch

from . import native

LINEARS = ["encoder.0", "encoder.3", "encoder.6", "mean_layer", "logvar_layer",
           "decoder.0", "decoder.3", "decoder.6", "decoder.9"]
BNS = ["encoder.1", "encoder.4", "encoder.7", "decoder.1", "decoder.4", "decoder.7"]


def param_specs(G, H, L):
    """(name, shape) in `model.parameters()` order (model.py:65-91)."""
    s = []
    for i, fan_in in enumerate([G, H, H]):
        s += [(f"encoder.{3*i}.weight", (H, fan_in)), (f"encoder.{3*i}.bias", (H,)),
              (f"encoder.{3*i+1}.weight", (H,)), (f"encoder.{3*i+1}.bias", (H,))]
    s += [("mean_layer.weight", (L, H)), ("mean_layer.bias", (L,)),
          ("logvar_layer.weight", (L, H)), ("logvar_layer.bias", (L,))]
    for i, fan_in in enumerate([L, H, H]):
        s += [(f"decoder.{3*i}.weight", (H, fan_in)), (f"decoder.{3*i}.bias", (H,)),
              (f"decoder.{3*i+1}.weight", (H,)), (f"decoder.{3*i+1}.bias", (H,))]
    s += [("decoder.9.weight", (G, H)), ("decoder.9.bias", (G,))]
    return s


def reference_init(G, H, L):
    """Host-side replay of the reference init on the global CPU generator: nn.Linear ctor
    (kaiming_uniform a=sqrt(5) weight, uniform(+-1/sqrt(fan_in)) bias, construction order), then
    xavier_uniform_ on every Linear weight and zero biases (model.py:115-120). BN: ones / zeros.
    Host work, once per model: not on the hot path."""
    shapes = dict(param_specs(G, H, L))
    P = {}
    for lin in LINEARS:
        w = torch.empty(shapes[lin + ".weight"])
        b = torch.empty(shapes[lin + ".bias"])
        torch.nn.init.kaiming_uniform_(w, a=math.sqrt(5))
        bound = 1.0 / math.sqrt(w.shape[1]) if w.shape[1] > 0 else 0.0
        torch.nn.init.uniform_(b, -bound, bound)
        P[lin + ".weight"], P[lin + ".bias"] = w, b
    for bn in BNS:
        P[bn + ".weight"] = torch.ones(H)
        P[bn + ".bias"] = torch.zeros(H)
    for lin in LINEARS:
        torch.nn.init.xavier_uniform_(P[lin + ".weight"])
        P[lin + ".bias"].zero_()
    return [P[n] for n, _ in param_specs(G, H, L)]


def _default_device():
    if not torch.cuda.is_available():
        raise RuntimeError("genome-minimizer-2 MI355X build: no HIP device visible (torch.cuda.is_available() "
                           "is False); the hot path has no CPU implementation")
    return torch.device("cuda", torch.cuda.current_device())


class VAE:
    """Drop-in for the reference VAE (model.py:13). `precision` selects the GEMM arithmetic of
    training/eval/encode (native.GM2_F32 exact fp32, native.GM2_BF16); sampling always decodes in
    exact fp32 so its thresholded masks match the fp32 reference."""

    def __init__(self, input_dim, hidden_dim, latent_dim, device=None, precision=native.GM2_BF16,
                 init=True):
        self.input_dim, self.hidden_dim, self.latent_dim = int(input_dim), int(hidden_dim), int(latent_dim)
        self.device = torch.device(device) if device is not None else None
        self.precision = precision
        self.training = True
        G, H, L = self.input_dim, self.hidden_dim, self.latent_dim
        self.specs = param_specs(G, H, L)
        self.offsets = native.param_offsets(G, H, L)
        self.n_params = self.offsets[-1]
        host = reference_init(G, H, L) if init else [torch.zeros(s) for _, s in self.specs]
        self._host_init = torch.cat([t.reshape(-1) for t in host])
        self.num_batches_tracked = [0] * 6
        self.params = None
        self.bn = None
        self._workspaces = {}
        self._shadow_stamp = {}
        self._version = 0
        if self.device is None or self.device.type == "cuda":
            self.to(self.device or _default_device())

    # ---------------------------------------------------------------- storage / torch-like API
    def to(self, device):
        device = torch.device(device)
        if device.type != "cuda":
            raise RuntimeError("the MI355X VAE lives on a HIP device; CPU execution is not provided")
        if self.params is None:
            self.params = self._host_init.to(device).contiguous()
            bn = torch.zeros(6, 2, self.hidden_dim)
            bn[:, 1] = 1.0
            self.bn = bn.to(device).contiguous()
            self._host_init = None
        else:
            self.params = self.params.to(device)
            self.bn = self.bn.to(device)
        self.device = device
        for prec, ws in self._workspaces.items():
            self._retire_workspace(ws, prec)
        self._workspaces.clear()
        self.touch()
        return self

    def touch(self):
        """Mark the fp32 master parameters as edited (GEMM shadows are re-derived lazily)."""
        self._version += 1

    def train(self, mode=True):
        self.training = bool(mode)
        return self

    def eval(self):
        return self.train(False)

    def param_views(self):
        out = OrderedDict()
        for i, (n, shp) in enumerate(self.specs):
            out[n] = self.params[self.offsets[i]:self.offsets[i + 1]].view(shp)
        return out

    def named_parameters(self):
        return list(self.param_views().items())

    def parameters(self):
        return list(self.param_views().values())

    def state_dict(self):
        """Same keys, order, shapes and dtypes as the reference module's state_dict."""
        views = self.param_views()
        sd = OrderedDict()
        for lin in ["encoder.0", "encoder.1", "encoder.3", "encoder.4", "encoder.6", "encoder.7",
                    "mean_layer", "logvar_layer", "decoder.0", "decoder.1", "decoder.3", "decoder.4",
                    "decoder.6", "decoder.7", "decoder.9"]:
            sd[lin + ".weight"] = views[lin + ".weight"].detach().clone()
            sd[lin + ".bias"] = views[lin + ".bias"].detach().clone()
            if lin in BNS:
                i = BNS.index(lin)
                sd[lin + ".running_mean"] = self.bn[i, 0].detach().clone()
                sd[lin + ".running_var"] = self.bn[i, 1].detach().clone()
                sd[lin + ".num_batches_tracked"] = torch.tensor(self.num_batches_tracked[i], dtype=torch.long)
        return sd

    def load_state_dict(self, sd, strict=True):
        views = self.param_views()
        expected = set(self.state_dict().keys()) if strict else set()
        missing = [k for k in expected if k not in sd]
        unexpected = [k for k in sd if strict and k not in expected]
        if missing or unexpected:
            raise RuntimeError(f"Error(s) in loading state_dict for VAE: missing {missing}, unexpected {unexpected}")
        with torch.no_grad():
            for k, v in sd.items():
                if k in views:
                    if tuple(v.shape) != tuple(views[k].shape):
                        raise RuntimeError(f"size mismatch for {k}: {tuple(v.shape)} vs {tuple(views[k].shape)}")
                    views[k].copy_(v.to(self.device, torch.float32))
                elif k.endswith("running_mean") or k.endswith("running_var"):
                    i = BNS.index(k.rsplit(".", 1)[0])
                    self.bn[i, 0 if k.endswith("mean") else 1].copy_(v.to(self.device, torch.float32))
                elif k.endswith("num_batches_tracked"):
                    self.num_batches_tracked[BNS.index(k.rsplit(".", 1)[0])] = int(v)
        self.touch()
        return self

    # ------------------------------------------------------------------ native workspaces
    def _retire_workspace(self, ws, prec):
        """An fp32 (sampling) workspace is about to be replaced or dropped: its decode counters
        start at zero in the next one, so its totals are kept on the host and decode_stats adds
        them back (whichever caller swapped it: a decode, an fp32 train/eval call, or `to`)."""
        if ws is not None and prec == native.GM2_F32:
            base = getattr(self, "_stats_base", {})
            self._stats_base = {k: base.get(k, 0) + ws.stat(v) for k, v in native.DECODE_STATS.items()}

    def workspace(self, prec, batch_max):
        """Workspace for (precision, capacity); reused while large enough."""
        key = prec
        ws = self._workspaces.get(key)
        if ws is None or ws.d.batch_max < batch_max:
            self._retire_workspace(ws, key)
            cap = max(int(batch_max), ws.d.batch_max if ws else 0)
            ws = native.Workspace(native.dims(self.input_dim, self.hidden_dim, self.latent_dim, cap), prec,
                                  self.device)
            self._workspaces[key] = ws
            self._shadow_stamp[key] = -1
        if self._shadow_stamp[key] != self._version:
            native.sync_shadows(ws, self.params)
            self._shadow_stamp[key] = self._version
        return ws

    def shadows_current(self, prec):
        """Called after an in-kernel optimizer step that updated the fp32 master AND refreshed the
        `prec` shadows itself: the parameters changed (new version), only that workspace is current."""
        self._version += 1
        if prec in self._workspaces:
            self._shadow_stamp[prec] = self._version

    # ---------------------------------------------------------------------- compute API
    # ------------------------------------------------------------- reference module surface
    def requires_grad_(self, flag=True):
        """Let torch autograd track the flat parameter buffer (VAE.forward's backward then writes
        dL/dtheta into self.params.grad, parameter views included)."""
        self.params.requires_grad_(flag)
        return self

    def zero_grad(self, set_to_none=True):
        self.params.grad = None

    def reparameterization(self, mean, logvar):
        """z = mean + exp(0.5*logvar) * randn_like(std) (model.py:100-104), on libgm2's kernel,
        differentiable (torch autograd) in mean and logvar."""
        eps = torch.randn_like(logvar)
        return _Reparam.apply(mean, logvar, eps)

    def forward(self, x, eps=None):
        """(x_hat, mean, logvar) = model(x) (model.py:109-113) through libgm2: encoder with
        BatchNorm in the module's train/eval mode (train mode updates the running statistics),
        reparameterisation (eps ~ N(0, I) drawn on the device like randn_like, unless given),
        decoder, sigmoid. x: a 0/1 tensor [B, G] (any dtype), a ResidentMatrix, or a
        (ResidentMatrix, int32 row-index tensor) pair. Differentiable under torch autograd in the
        parameters (self.params, after requires_grad_()) through gm2_backward_outputs, so
        arbitrary LossComponents can be trained on it (trainer.py:349-352)."""
        from .data import ResidentMatrix
        if isinstance(x, tuple):
            mat, rows = x
        else:
            mat, rows = (x if isinstance(x, ResidentMatrix) else ResidentMatrix(x, device=self.device)), None
        n = int(rows.shape[0]) if rows is not None else mat.n
        if self.training and n < 2:
            raise ValueError(f"Expected more than 1 value per channel when training, got input size [1, {self.hidden_dim}]")
        if eps is None:
            eps = torch.randn(n, self.latent_dim, device=self.device)
        eps = eps.to(self.device, torch.float32).contiguous()
        out = _Forward.apply(self.params, self, mat, rows, n, eps)
        if self.training:
            self.num_batches_tracked = [k + 1 for k in self.num_batches_tracked]
        return out

    __call__ = forward

    def decode(self, z):
        """p = sigmoid(decoder(z)) (model.py:106-107), exact fp32. Eval mode (running statistics):
        every reference call site decodes a loaded, eval()'d model (extras.py:185-198)."""
        if self.training:
            raise RuntimeError("VAE.decode on this build runs eval-mode BatchNorm; call model.eval() first "
                               "(train-mode decoding runs inside model(x))")
        _, p = self.decode_mask(z, want_probs=True)
        return p

    def decode_mask(self, z, want_probs=False, chunk=65536):
        """(mask u8 [N,G], probs fp32 [N,G] or None) = (sigmoid(decode(z)) > 0.5, p).
        Eval-mode BatchNorm (running statistics), exactly as model.decode after model.eval()."""
        z = z.to(self.device, torch.float32).contiguous()
        N, G = z.shape[0], self.input_dim
        mask = torch.empty(N, G, dtype=torch.uint8, device=self.device)
        probs = torch.empty(N, G, dtype=torch.float32, device=self.device) if want_probs else None
        for s in range(0, N, chunk):
            n = min(chunk, N - s)
            ws = self.workspace(native.GM2_F32, min(chunk, N))
            native.decode_mask(ws, self.params, self.bn, z[s:s + n], n, mask[s:], G,
                               None if probs is None else probs[s:], G)
        return mask, probs

    def decode_bits(self, z, want_probs=False, chunk=65536):
        """Like decode_mask, but the masks stay on the device packed 8 genes per byte
        (gm2.masks.PackedMasks): what --mode sample hands to the mask consumers."""
        from .masks import PackedMasks
        z = z.to(self.device, torch.float32).contiguous()
        N, G = z.shape[0], self.input_dim
        pm = PackedMasks.empty(N, G, self.device)
        probs = torch.empty(N, G, dtype=torch.float32, device=self.device) if want_probs else None
        for s in range(0, N, chunk):
            n = min(chunk, N - s)
            ws = self.workspace(native.GM2_F32, min(chunk, N))
            native.decode_bits(ws, self.params, self.bn, z[s:s + n], n, pm.bits[s:], pm.ld,
                               None if probs is None else probs[s:], G)
        return pm, probs

    def decode_stats(self):
        """The sampling decodes' counters on this model's fp32 (sampling) workspace, cumulative
        (gm2.h GM2_STAT_*): decodes and output-layer tiles per path (bf16x3 split / exact fp32),
        logits of the certified band recomputed in fp64, the mask bits that recompute flipped,
        band elements beyond a call's list capacity and the 256 x 256 blocks recomputed whole in fp64
        for them. Zeros before the first decode; monotone across workspace replacements. Waits for
        the device."""
        ws = self._workspaces.get(native.GM2_F32)
        base = getattr(self, "_stats_base", {})
        return {k: base.get(k, 0) + (ws.stat(v) if ws is not None else 0) for k, v in native.DECODE_STATS.items()}

    def encode(self, x):
        """(mean, logvar) of the eval-mode encoder (model.py:95-98) for a 0/1 matrix x [B, G]
        (every reference call site encodes an eval()'d model: extras.py:205-228)."""
        from .data import ResidentMatrix
        m = x if isinstance(x, ResidentMatrix) else ResidentMatrix(x, device=self.device)
        B = m.n
        mu = torch.empty(B, self.latent_dim, device=self.device)
        lv = torch.empty(B, self.latent_dim, device=self.device)
        ws = self.workspace(self.precision, B)
        native.encode(ws, native.make_batch(m.data, m.ld, None, B, None), self.params, self.bn, mu, lv)
        return mu, lv

    def __repr__(self):
        return (f"VAE(input_dim={self.input_dim}, hidden_dim={self.hidden_dim}, latent_dim={self.latent_dim}, "
                f"device={self.device}, precision={'fp32' if self.precision == native.GM2_F32 else 'bf16'})")


class _Forward(torch.autograd.Function):
    """model(x) on libgm2 with a libgm2 backward (gm2_forward / gm2_backward_outputs). The
    workspace keeps the forward's activations; any later call that runs on the same workspace
    (forward, encode, eval, decode, recon counts, training) invalidates them: the backward checks
    the workspace's generation counter and raises."""

    @staticmethod
    def forward(ctx, params, model, mat, rows, n, eps):
        dev = model.device
        G, L = model.input_dim, model.latent_dim
        ws = model.workspace(model.precision, n)
        probs = torch.empty(n, G, device=dev)
        mu = torch.empty(n, L, device=dev)
        lv = torch.empty(n, L, device=dev)
        batch = native.make_batch(mat.data, mat.ld, rows, n, eps)
        native.forward(ws, batch, params.detach(), model.bn, int(model.training), probs, G, mu, lv)
        ctx.model, ctx.mat, ctx.rows, ctx.n, ctx.train = model, mat, rows, n, model.training
        ctx.ws, ctx.gen = ws, ws.gen
        ctx.save_for_backward(probs, eps)
        return probs, mu, lv

    @staticmethod
    def backward(ctx, dprobs, dmu, dlv):
        m = ctx.model
        if m._workspaces.get(m.precision) is not ctx.ws or ctx.ws.gen != ctx.gen:
            raise RuntimeError("VAE.forward activations were overwritten by a later call on the same model's "
                               "workspace (forward, encode, eval, decode or training); call backward first")
        probs, eps = ctx.saved_tensors
        if dprobs is None:
            dprobs = torch.zeros_like(probs)
        grads = torch.empty_like(m.params)
        ws = ctx.ws
        batch = native.make_batch(ctx.mat.data, ctx.mat.ld, ctx.rows, ctx.n, eps)
        native.backward_outputs(ws, batch, m.params.detach(), int(ctx.train), probs, m.input_dim,
                                dprobs.contiguous(), None if dmu is None else dmu.contiguous(),
                                None if dlv is None else dlv.contiguous(), grads)
        return grads, None, None, None, None, None


class _Reparam(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mean, logvar, eps):
        mean, logvar, eps = (t.contiguous().float() for t in (mean, logvar, eps))
        z = torch.empty_like(mean)
        native.reparameterize(mean.numel(), mean, logvar, eps, z)
        ctx.save_for_backward(mean, logvar, eps)
        return z

    @staticmethod
    def backward(ctx, dz):
        mean, logvar, eps = ctx.saved_tensors
        dmu, dlv = torch.empty_like(mean), torch.empty_like(mean)
        native.reparameterize(mean.numel(), mean, logvar, eps, None, dz.contiguous(), dmu, dlv)
        return dmu, dlv, None
