"""CPU-side checks of the device-op reference math (the same formulas the HIP kernels implement)."""
import torch

from spark_rapids_ml_nai_amd import ops


def test_split_bf16x3_exact_and_distance():
    g = torch.Generator().manual_seed(0)
    m, n, k = 300, 70, 40
    C = torch.randn(k, n, generator=g) * 3
    X = (C[torch.randint(0, k, (m,), generator=g)] + 0.3 * torch.randn(m, n, generator=g)).float()
    P = ops.split_bf16x3(X)
    assert P.dtype == torch.bfloat16 and P.shape == (3, 384, 80)
    # three bf16 pieces carry all 24 significand bits of fp32
    assert torch.equal(P.float().sum(0)[:m, :n], X)
    xn = (X * X).sum(1)
    lab_s, d_s = ops.nearest_centroid_split(P, m, C, xn)
    lab, d = ops.nearest_centroid(X, C, xn)
    D = torch.cdist(X.double(), C.double()) ** 2
    ref_d = D.min(1).values
    assert torch.all(D[torch.arange(m), lab_s.long()] <= ref_d + 1e-4 * (1 + ref_d))
    torch.testing.assert_close(d_s.double(), ref_d, rtol=1e-4, atol=1e-3)


def test_parse_cpulist_and_numa_bind_noop_on_cpu():
    import torch

    from spark_rapids_ml_nai_amd.parallel.context import _parse_cpulist, bind_numa_local

    assert _parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert bind_numa_local(torch.device("cpu")) is None


def test_sorted_counts_matches_bincount():
    """Label counts by binary search over sorted labels (cluster sums, IVF lists, UMAP CSR) equal
    torch.bincount, including empty labels at both ends and in the middle."""
    import torch

    from spark_rapids_ml_nai_amd import ops

    g = torch.Generator().manual_seed(3)
    for k in (1, 7, 1000):
        lab = torch.randint(0, k, (5000,), generator=g)
        lab = lab[(lab != k // 2) | (k == 1)]  # a gap
        s, _ = torch.sort(lab)
        assert torch.equal(ops.sorted_counts(s, k), torch.bincount(lab, minlength=k))
    s32 = torch.tensor([1, 1, 4], dtype=torch.int32)
    assert ops.sorted_counts(s32, 6).tolist() == [0, 2, 0, 0, 1, 0]
