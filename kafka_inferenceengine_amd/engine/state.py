"""Device-resident Kalman state: SoA mean ``x[n_p, ld]`` and packed symmetric
blocks ``P[n_p(n_p+1)/2, ld]`` (precision or covariance).

Replaces the reference's interleaved vector + (n_p·N)² sparse matrices
(``linear_kf.py:171``, ``kf_tools.py:131``).  Conversions to/from the
reference representation are provided for the compatibility paths.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import scipy.sparse as sp
import torch

from ..utils.blocks import (LazyBlockDiag, interleaved_to_soa, ntri, pack_blocks, pack_matrix, soa_to_interleaved,
                            sparse_to_blocks)

PRECISION = "precision"
COVARIANCE = "covariance"


@dataclass
class KFState:
    x: torch.Tensor          # [n_p, ld] float32
    P: torch.Tensor          # [ntri, ld] float32 (packed upper triangle)
    kind: str                # PRECISION | COVARIANCE
    N: int                   # active pixels (<= ld)
    # packed rows of P that hold values (bit t: row t); None = all.  An analysis
    # under EngineConfig.store_precision="auto" stores only what the next
    # forecast reads (the LAI propagator: one diagonal entry, kf_tools.py:292-314)
    p_valid: int | None = None
    # COVARIANCE states only: the p_valid rows tri(j, j) hold the analysis
    # PRECISION diagonal (P^-1)_jj -- what the gain form's stored-rows policy
    # keeps for the next fused forecast (GainArgs.pdiag_rows / PropArgs.pa_pdiag)
    p_diag_precision: bool = False

    @property
    def full(self) -> bool:
        return self.p_valid is None

    def require_full(self, what: str = "this operation"):
        if self.p_valid is not None:
            rows = [t for t in range(self.P.shape[0]) if (self.p_valid >> t) & 1]
            raise RuntimeError(f"{what} needs the full packed {self.kind}, but this analysis stored rows {rows} only "
                               "(EngineConfig.store_precision='auto' keeps what the next forecast reads); set "
                               "store_precision='always' or read the state of the run's last date")

    @property
    def n_params(self) -> int:
        return int(self.x.shape[0])

    @property
    def device(self):
        return self.x.device

    def clone(self) -> "KFState":
        return KFState(self.x.clone(), self.P.clone(), self.kind, self.N, self.p_valid, self.p_diag_precision)

    def copy_(self, other: "KFState") -> "KFState":
        self.x.copy_(other.x)
        self.P.copy_(other.P)
        self.kind = other.kind
        self.p_valid = other.p_valid
        self.p_diag_precision = other.p_diag_precision
        return self

    @classmethod
    def empty(cls, n_params, N, device, kind=PRECISION, ld=None) -> "KFState":
        ld = N if ld is None else ld
        x = torch.zeros((n_params, ld), dtype=torch.float32, device=device)
        P = torch.zeros((ntri(n_params), ld), dtype=torch.float32, device=device)
        return cls(x, P, kind, N)

    @classmethod
    def constant(cls, mean, mat, N, device, kind=PRECISION) -> "KFState":
        """Every pixel = (mean, mat) — e.g. a prior.  Built on the device."""
        mean = np.asarray(mean, dtype=np.float64)
        n = mean.size
        s = cls.empty(n, N, device, kind)
        s.x.copy_(torch.from_numpy(mean.astype(np.float32))[:, None].expand(n, N))
        s.P.copy_(torch.from_numpy(pack_matrix(np.asarray(mat)).astype(np.float32))[:, None].expand(-1, N))
        return s

    # ------------------------------------------------- reference interop
    @classmethod
    def from_reference(cls, x_flat, P_mat, n_params, kind, device, pixel_slice=None) -> "KFState":
        """Interleaved vector + block-diagonal matrix (sparse/dense/None) -> state.

        ``pixel_slice`` selects this rank's pixels (global -> local)."""
        x = interleaved_to_soa(np.asarray(x_flat, dtype=np.float64), n_params)
        if pixel_slice is not None:
            x = x[:, pixel_slice]
        N = x.shape[1]
        if P_mat is None:
            packed = np.zeros((ntri(n_params), N))
        elif isinstance(P_mat, LazyBlockDiag):
            packed = P_mat.packed
            if pixel_slice is not None:
                packed = packed[:, pixel_slice]
        else:
            if pixel_slice is not None and sp.issparse(P_mat):
                sl = np.arange(P_mat.shape[0]).reshape(-1, n_params)[pixel_slice].ravel()
                P_mat = sp.csr_matrix(P_mat)[sl][:, sl]
            blocks = sparse_to_blocks(P_mat, n_params, check=True)
            if pixel_slice is not None and not sp.issparse(P_mat):
                blocks = blocks[pixel_slice]
            packed = pack_blocks(blocks)
        xt = torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).to(device)
        Pt = torch.from_numpy(np.ascontiguousarray(packed, dtype=np.float32)).to(device)
        return cls(xt, Pt, kind, N)

    def to_reference(self):
        """(x_flat numpy, LazyBlockDiag of P) — the reference's (x, P / P^-1)."""
        self.require_full("to_reference")
        x = self.x[:, :self.N].detach().cpu().numpy().astype(np.float64)
        P = self.P[:, :self.N].detach().cpu().numpy()
        return soa_to_interleaved(x), LazyBlockDiag(P, self.n_params)

    def numpy(self):
        self.require_full("numpy")
        return (self.x[:, :self.N].detach().cpu().numpy(), self.P[:, :self.N].detach().cpu().numpy())


class LazyForecast:
    """A forecast that has not been written to memory: the previous analysis
    plus the propagation arguments.  The fused analysis kernel evaluates it per
    pixel (``AnalysisArgs.prop``); every other consumer calls
    :meth:`materialize`, which runs the propagate kernel."""

    kind = PRECISION

    def __init__(self, src: KFState, spec: dict, blend_pix, q_pix, materialize, kind=PRECISION, cache=None):
        self.src, self.spec, self.blend_pix, self.q_pix = src, spec, blend_pix, q_pix
        self._materialize = materialize
        self._cache = cache  # engine dict: content key -> (PropArgs, device copy)
        self.kind = kind     # form of the forecast it stands for (COVARIANCE: gain-form K1g consumer)

    @property
    def N(self) -> int:
        return self.src.N

    @property
    def n_params(self) -> int:
        return self.src.n_params

    @property
    def device(self):
        return self.src.device

    def _key(self, bm, bc):
        import numpy as np

        def v(x):
            return np.asarray(x).tobytes() if not isinstance(x, (int, float, bool, str)) else x
        ptr = lambda t: 0 if t is None else t.data_ptr()   # noqa: E731
        head = (ptr(self.src.x), ptr(self.src.P), self.N, self.src.x.shape[1], ptr(self.q_pix), ptr(bm), ptr(bc),
                str(self.src.x.device), bool(self.src.p_diag_precision))
        if "_key" in self.spec:        # memoised argument dict (LinearKalman.advance_state)
            return head + (self.spec["_key"],)
        return head + tuple((k, v(x)) for k, x in sorted(self.spec.items()))

    def handle(self):
        """Fused-propagation arguments; the packed device block is reused across
        dates whose analysis buffers and propagation parameters coincide (the
        block holds only addresses and parameters)."""
        from ..ops import kernels as K
        bm, bc = self.blend_pix if self.blend_pix else (None, None)
        key = None
        if self._cache is not None:
            key = self._key(bm, bc)
            hit = self._cache.get(key)
            if hit is not None:
                self._cache["_hits"] = self._cache.get("_hits", 0) + 1
                h = K.PropHandle(hit[0], self.src.x.device, (self.src.x, self.src.P), fused=True)
                h._buf = hit[1]
                return h
        h = K.prop_args(self.n_params, self.spec, self.src.x, self.src.P, N=self.N, q_pix=self.q_pix,
                        blend_mean_pix=bm, blend_cinv_pix=bc, fused=True, pa_pdiag=self.src.p_diag_precision)
        if key is not None:
            self._cache["_misses"] = self._cache.get("_misses", 0) + 1
            if len(self._cache) >= 256:
                for k in [k for k in self._cache if not isinstance(k, str)][:64]:
                    del self._cache[k]
            self._cache[key] = (h.args, h.device_copy())
        return h

    def materialize(self) -> KFState:
        return self._materialize()
