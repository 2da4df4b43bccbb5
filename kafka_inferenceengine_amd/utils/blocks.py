"""Per-pixel block helpers: the bridge between the reference's global sparse
matrices and this framework's packed SoA layout.

The reference stores the state as one interleaved vector ``[p0θ0 … p0θ(n-1),
p1θ0, …]`` (``kafka/inference/kf_tools.py:301-303``) and precision/covariance
as an (n_p·N)² block-diagonal scipy matrix (``kf_tools.py:131``,
``utils.py:240-339``).  Here a state is ``x[n_p, N]`` (SoA) and a symmetric
block set is the packed upper triangle ``P[n_p(n_p+1)/2, N]`` in row-major
order — the exact layout the gfx950 kernels read (``csrc/kf_core.h`` ``tri``).
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp


def ntri(n: int) -> int:
    return n * (n + 1) // 2


def tri_indices(n: int) -> tuple[np.ndarray, np.ndarray]:
    """Row/col index of each packed slot (row-major upper triangle)."""
    iu, ju = [], []
    for i in range(n):
        for j in range(i, n):
            iu.append(i)
            ju.append(j)
    return np.array(iu), np.array(ju)


def tri_pos(n: int, i: int, j: int) -> int:
    if i > j:
        i, j = j, i
    return i * n - (i * (i - 1)) // 2 + (j - i)


def pack_blocks(blocks: np.ndarray) -> np.ndarray:
    """[N, n, n] symmetric blocks -> packed [ntri(n), N]."""
    blocks = np.asarray(blocks)
    n = blocks.shape[-1]
    iu, ju = tri_indices(n)
    return np.ascontiguousarray(blocks[:, iu, ju].T)


def unpack_blocks(packed: np.ndarray, n: int) -> np.ndarray:
    """Packed [ntri(n), N] -> symmetric [N, n, n]."""
    packed = np.asarray(packed)
    N = packed.shape[1]
    iu, ju = tri_indices(n)
    out = np.zeros((N, n, n), dtype=packed.dtype)
    out[:, iu, ju] = packed.T
    out[:, ju, iu] = packed.T
    return out


def pack_matrix(m: np.ndarray) -> np.ndarray:
    """One symmetric n x n matrix -> packed vector."""
    m = np.asarray(m)
    iu, ju = tri_indices(m.shape[0])
    return m[iu, ju].copy()


def unpack_matrix(v: np.ndarray, n: int) -> np.ndarray:
    iu, ju = tri_indices(n)
    m = np.zeros((n, n), dtype=np.asarray(v).dtype)
    m[iu, ju] = v
    m[ju, iu] = v
    return m


def interleaved_to_soa(x: np.ndarray, n_params: int) -> np.ndarray:
    """Reference flat state (pixel-major, interleaved) -> x[n_params, N]."""
    x = np.asarray(x).ravel()
    return np.ascontiguousarray(x.reshape(-1, n_params).T)


def soa_to_interleaved(x: np.ndarray) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(x).T).ravel()


def blocks_to_sparse(blocks: np.ndarray, fmt: str = "csr", dtype=None) -> sp.spmatrix:
    """[N, n, n] -> block-diagonal sparse matrix, built without Python loops."""
    blocks = np.asarray(blocks, dtype=dtype)
    N, n, _ = blocks.shape
    if N == 0:
        return sp.csr_matrix((0, 0), dtype=blocks.dtype)
    indptr = np.arange(N + 1)
    indices = np.arange(N)
    m = sp.bsr_matrix((blocks, indices, indptr), shape=(N * n, N * n))
    return m.asformat(fmt)


def sparse_to_blocks(m, n: int, check: bool = True) -> np.ndarray:
    """Block-diagonal sparse (or dense) matrix -> [N, n, n] blocks.

    Raises ``ValueError`` when ``check`` and a non-zero lies outside the
    n x n diagonal blocks (i.e. the matrix couples pixels).
    """
    if not sp.issparse(m):
        m = sp.csr_matrix(np.asarray(m))
    m = m.tocoo()
    size = m.shape[0]
    if size % n:
        raise ValueError(f"matrix of size {size} is not a multiple of n_params={n}")
    N = size // n
    r, c, v = m.row, m.col, m.data
    inblk = (r // n) == (c // n)
    if check and not np.all(inblk | (v == 0)):
        raise ValueError("matrix is not block diagonal with n_params blocks")
    out = np.zeros((N, n, n), dtype=np.result_type(v.dtype, np.float32))
    np.add.at(out, (r[inblk] // n, r[inblk] % n, c[inblk] % n), v[inblk])
    return out


def block_diag_dense(blocks: np.ndarray) -> np.ndarray:
    N, n, _ = blocks.shape
    out = np.zeros((N * n, N * n), dtype=blocks.dtype)
    for i in range(N):
        out[i * n:(i + 1) * n, i * n:(i + 1) * n] = blocks[i]
    return out


class LazyBlockDiag:
    """Read-only stand-in for the reference's block-diagonal ``P_analysis_inverse``
    handed to legacy ``dump_data`` writers: supports ``diagonal()``,
    ``todense()``, ``tocsr()`` and ``shape`` without materialising N²."""

    def __init__(self, packed: np.ndarray, n: int):
        self.packed = np.asarray(packed)
        self.n = n
        self.N = self.packed.shape[1]
        self.shape = (self.N * n, self.N * n)

    def diagonal(self) -> np.ndarray:
        d = np.empty(self.N * self.n, dtype=self.packed.dtype)
        for j in range(self.n):
            d[j::self.n] = self.packed[tri_pos(self.n, j, j)]
        return d

    def blocks(self) -> np.ndarray:
        return unpack_blocks(self.packed, self.n)

    def tocsr(self):
        return blocks_to_sparse(self.blocks(), "csr")

    def todense(self):
        return self.tocsr().todense()

    def __mul__(self, other):
        if np.isscalar(other):
            return LazyBlockDiag(self.packed * other, self.n)
        return NotImplemented
