"""Hessian calibration on the HIP device.

The reference computes the activation second moment that `caldera()` weights its error by
in its driver (`main.py:268-319`): a forward hook stores each Linear layer's input
(`hook_fn`, main.py:50-51, `inputs[0].detach().cpu()`), and after every calibration sample
the driver forms `a_aT = A A^T` in float64 from `activations.view(D, -1)` (main.py:302-305),
adds it to a running sum and divides the sum by `idx + 1` (main.py:307).  The file it ships
(`diag_Hessians.pt`) holds the per-layer diagonal (float64, keyed by module name, read as
`Hall[name]` at main.py:163).

`HessianCalibrator` keeps the activations on the device (no per-call host copy) and
accumulates through the HIP library:
  * diagonal: `cq_act_sqsum_cols` / `cq_act_sqsum_rows` (HBM-bound streaming fp64
    reductions, deterministic order);
  * full Hessian: `cq_gram_f64` (fp64 MFMA Gram, the kernel the solver uses).
Two modes:
  * ``"reference"`` — main.py's arithmetic exactly: only the LAST forward input of each
    sample is used (the hook overwrites `layer_activations[name]`, so under `generate()` it
    is the final decode step), reshaped with `.view(D, -1)` (a reshape of token-major
    memory, not a transpose), and the running sum is divided by `idx + 1` after every
    sample (`end_sample()`);
  * ``"mean"`` (default) — the second moment the reference means to compute: every forward
    call's tokens, sum of a a^T over tokens / token count.
"""
from __future__ import annotations

import torch

from . import _lib as K


class HessianCalibrator:
    """Forward hooks accumulating per-layer activation second moments on the HIP device.

    model: any torch.nn.Module on a HIP device.  names: module names to hook (default: every
    `module_types` module, main.py:271-274 hooks every nn.Linear).  full: also (or only,
    with diag=False) the dense D x D Hessian (main.py's `a_aT`); diag: the diagonal that
    diag_Hessians.pt ships."""

    def __init__(self, model: torch.nn.Module, names=None, *, mode: str = "mean", full: bool = False,
                 diag: bool = True, module_types=(torch.nn.Linear,)):
        if mode not in ("mean", "reference"):
            raise ValueError(f"mode must be 'mean' or 'reference', got {mode!r}")
        if not (full or diag):
            raise ValueError("nothing to accumulate: full=False and diag=False")
        self.model, self.mode, self.full, self.diag = model, mode, full, diag
        mods = dict(model.named_modules())
        if names is None:
            names = [n for n, m in mods.items() if isinstance(m, module_types)]
        missing = [n for n in names if n not in mods]
        if missing:
            raise KeyError(f"no such modules: {missing[:4]}")
        self.names = list(names)
        self._mods = {n: mods[n] for n in self.names}
        self._handles = []
        self._diag: dict[str, torch.Tensor] = {}
        self._full: dict[str, torch.Tensor] = {}
        self._tokens: dict[str, int] = {}
        self._last: dict[str, torch.Tensor] = {}
        self.samples = 0

    # ------------------------------------------------------------------ hooks
    def attach(self):
        if not self._handles:
            for n, m in self._mods.items():
                self._handles.append(m.register_forward_hook(
                    lambda mod, inp, out, name=n: self._on_forward(name, inp)))
        return self

    def detach(self):
        for h in self._handles:
            h.remove()
        self._handles = []

    def __enter__(self):
        return self.attach()

    def __exit__(self, *exc):
        self.detach()

    def _on_forward(self, name, inputs):
        a = inputs[0].detach()
        if a.device.type != "cuda":
            raise RuntimeError("HessianCalibrator: activations must live on the HIP device")
        if self.mode == "reference":
            self._last[name] = a  # main.py:51 overwrites: only the last call of a sample counts
            return
        X = a.reshape(-1, a.shape[-1])
        self._accumulate(name, X, rows_are_tokens=True, post=1.0)
        self._tokens[name] = self._tokens.get(name, 0) + X.shape[0]

    # ------------------------------------------------------------------ accumulation
    def _accumulate(self, name, X, *, rows_are_tokens: bool, post: float):
        """rows_are_tokens: X (T, D), H += X^T X; else X (D, L), H += X X^T (then * post)."""
        D = X.shape[1] if rows_are_tokens else X.shape[0]
        dev = X.device
        if self.diag:
            acc = self._diag.get(name)
            fresh = acc is None
            if fresh:
                acc = self._diag[name] = torch.empty(D, dtype=torch.float64, device=dev)
            if rows_are_tokens:
                K.act_sqsum_cols(X, acc, accumulate=not fresh, post=post)
            else:
                K.act_sqsum_rows(X, acc, accumulate=not fresh, post=post)
        if self.full:
            X32 = X if X.dtype == torch.float32 else X.float()
            X32 = X32.contiguous()
            if rows_are_tokens:  # C = A^T B, A = B = X (K = T rows)
                G = K.gram_f64(X32, X32)[0]
            else:                # C = X X^T: A, B stored M x K (trans)
                G = K.gram_f64(X32, X32, ta=True, tb=True)[0]
            acc = self._full.get(name)
            if acc is None:
                self._full[name] = G if post == 1.0 else G.mul_(post)
            else:
                acc.add_(G)
                if post != 1.0:
                    acc.mul_(post)

    def end_sample(self):
        """Close one calibration sample (main.py:296-308): in reference mode, fold each
        layer's last forward input as `view(D, -1)` and apply the running `/ (idx + 1)` to
        every accumulated layer; in mean mode only counts samples."""
        idx = self.samples
        self.samples += 1
        if self.mode != "reference":
            return
        post = 1.0 / (idx + 1)
        for name in self.names:
            a = self._last.pop(name, None)
            if a is not None:
                if a.dim() != 3:
                    raise ValueError(f"{name}: reference mode expects (batch, tokens, D) inputs, got {tuple(a.shape)}")
                D = a.shape[2]
                self._accumulate(name, a.reshape(D, -1), rows_are_tokens=False, post=post)
            else:  # no new term this sample: the running division still applies
                if name in self._diag:
                    self._diag[name].mul_(post)
                if name in self._full:
                    self._full[name].mul_(post)

    # ------------------------------------------------------------------ results
    def hessians(self, full: bool | None = None) -> dict[str, torch.Tensor]:
        """{name: fp64 diagonal (D,)} (or the dense (D, D) with full=True), on the device."""
        want_full = self.full and not self.diag if full is None else full
        src = self._full if want_full else self._diag
        if want_full and not self.full:
            raise ValueError("calibrator was built with full=False")
        if not want_full and not self.diag:
            raise ValueError("calibrator was built with diag=False")
        out = {}
        for name in self.names:
            if name not in src:
                continue
            t = src[name]
            if self.mode == "mean":
                t = t / max(self._tokens.get(name, 0), 1)
            out[name] = t
        return out

    def save(self, path: str, full: bool | None = None):
        """torch.save of {name: fp64 tensor} on the host — the diag_Hessians.pt layout."""
        torch.save({k: v.cpu() for k, v in self.hessians(full).items()}, path)
