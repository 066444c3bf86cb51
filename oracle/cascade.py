"""numpy restatement of the two PyTorch-CPU reductions whose ORDER fixes the soft
resampler's indices bit for bit -- TEST INFRASTRUCTURE ONLY.

The reference's ``soft_resampler`` (resamplers.py:20-60) calls ``torch.sum`` and
``torch.cumsum`` on CPU float32 rows.  Those kernels live in a third-party
dependency (PyTorch ATen; the reference pins torch==1.9.0 in requirements.txt:1,
this container -- and the GPU box -- run torch 2.10.0):

* ``torch.sum(x, dim=-1)`` on a contiguous float32 row is ATen's *cascade sum*
  (aten/src/ATen/native/cpu/SumKernel.cpp): the row is read as 8-float vectors
  (``Vectorized<float>`` is 32 bytes in the DEFAULT/AVX2 builds and the sum stub
  has no AVX512 variant), the vectors are dealt round robin into 4 ILP
  accumulators, each accumulator is a 4-level cascade whose level step is
  ``2 ** max(4, ceil_log2(n_vec // 4) // 4)``; leftover vectors go into ILP slot 0,
  the 4 slots are folded, the scalar tail (n % 8 elements) is summed first and
  the 8 lanes are then added in lane order.  Rows shorter than 8 go through the
  same cascade with scalar "vectors" of width 1.
* ``torch.cumsum`` on float32 accumulates in float64 and rounds each prefix to
  float32.

``tests/test_cascade.py`` pins both against torch on random rows of many
lengths.  The HIP soft-resampler kernel implements exactly this order
(``csrc/resample_soft.hip``).
"""
import numpy as np

f32 = np.float32


def ceil_log2(n: int) -> int:
    return 0 if n <= 1 else int(n - 1).bit_length()


def _multi_row_sum(rows: np.ndarray, size: int) -> np.ndarray:
    """Cascade over ``size`` leading rows of ``rows`` (size, 4, W) -> (4, W) float32."""
    levels = 4
    power = max(4, ceil_log2(size) // levels)
    step = 1 << power
    mask = step - 1
    acc = np.zeros((levels,) + rows.shape[1:], dtype=f32)
    i = 0
    while i + step <= size:
        for j in range(step):
            acc[0] = (acc[0] + rows[i + j]).astype(f32)
        i += step
        for j in range(1, levels):
            acc[j] = (acc[j] + acc[j - 1]).astype(f32)
            acc[j - 1] = 0
            if i & (mask << (j * power)):
                break
    while i < size:
        acc[0] = (acc[0] + rows[i]).astype(f32)
        i += 1
    for j in range(1, levels):
        acc[0] = (acc[0] + acc[j]).astype(f32)
    return acc[0]


def _row_sum(vecs: np.ndarray) -> np.ndarray:
    """row_sum over ``vecs`` (n, W): ILP-4 cascade then fold -> (W,)."""
    n = vecs.shape[0]
    n4 = n // 4
    if n4 > 0:
        ps = _multi_row_sum(vecs[: n4 * 4].reshape(n4, 4, -1), n4).copy()
    else:
        ps = np.zeros((4,) + vecs.shape[1:], dtype=f32)
    for i in range(n4 * 4, n):
        ps[0] = (ps[0] + vecs[i]).astype(f32)
    for k in range(1, 4):
        ps[0] = (ps[0] + ps[k]).astype(f32)
    return ps[0]


def torch_cpu_row_sum(x: np.ndarray) -> np.float32:
    """Bit-exact float32 ``torch.sum(x)`` for a contiguous CPU row (see module doc)."""
    x = np.ascontiguousarray(x, dtype=f32)
    n = x.shape[0]
    V = 8
    if n < V:
        return f32(_row_sum(x.reshape(n, 1))[0])
    nv = n // V
    lanes = _row_sum(x[: nv * V].reshape(nv, V))
    acc = f32(0)
    for k in range(nv * V, n):
        acc = f32(acc + x[k])
    for k in range(V):
        acc = f32(acc + lanes[k])
    return acc


def torch_cpu_cumsum(x: np.ndarray) -> np.ndarray:
    """float32 ``torch.cumsum`` on CPU: float64 running sum, rounded per prefix."""
    return np.cumsum(np.asarray(x, dtype=np.float64)).astype(f32)
