"""Pin oracle/cascade.py (the reduction order the HIP soft resampler implements)
against torch's own CPU kernels."""
import numpy as np
import pytest
import torch

from oracle.cascade import torch_cpu_cumsum, torch_cpu_row_sum

SIZES = [1, 2, 3, 5, 7, 8, 9, 15, 16, 31, 32, 33, 63, 64, 65, 100, 127, 128, 129, 255, 256, 257,
         500, 1000, 1023, 1024, 1025, 2048, 4000, 4096, 5000, 10000, 16385, 40000]


@pytest.mark.parametrize("n", SIZES)
def test_row_sum_matches_torch(n):
    rng = np.random.default_rng(n)
    x = (rng.random((3, n)) * np.exp(rng.normal(size=(3, n)) * 3)).astype(np.float32)
    ref = torch.from_numpy(x).sum(dim=-1).numpy()
    for b in range(3):
        assert torch_cpu_row_sum(x[b]) == ref[b]


@pytest.mark.parametrize("n", [1, 7, 100, 1000, 10000])
def test_cumsum_matches_torch(n):
    rng = np.random.default_rng(n + 1)
    x = rng.random((2, n)).astype(np.float32)
    ref = torch.cumsum(torch.from_numpy(x), dim=1).numpy()
    for b in range(2):
        np.testing.assert_array_equal(torch_cpu_cumsum(x[b]), ref[b])
