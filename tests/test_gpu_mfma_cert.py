"""Pin the hardware assumption under the bf16 GEMM-form certificate (knn_capi.cpp
certificate(), DESIGN.md "Certificate"): on v_mfma_f32_32x32x16_bf16, bf16 x bf16
products are exact and the MFMA's internal sums err by no more than 2u (u = 2^-24) per
addition, plus at most 2^-126 per operation where denormal values are flushed.  Then the
dot product of K products p_i satisfies

    |mfma - sum p_i| <= 2 u K sum |p_i| + K 2^-126,

which is the dot term the filter's coef = (6d+32) u and eta = (6d+8) 2^-125 cover.  The
probe (knn_mfma_probe_bf16) runs the filter's own MFMA chain and lane map; the exact sum
comes from math.fsum over float64 products (exact: bf16 x bf16 has 16 significant bits).
Also bf16-data stress cases for KNN_ALGO_GEMM (bf16 data on the bf16 MFMA), mirroring
test_split_operands_stress for the fp32 filters.
"""
import math
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

U = 2.0 ** -24


def _bf16(x):
    """float64 array -> bf16 bits (round to nearest even) and the exact float64 values."""
    f = np.asarray(x, np.float32)
    u = f.view(np.uint32).astype(np.uint64)
    bits = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    vals = (bits.astype(np.uint32) << 16).view(np.float32).astype(np.float64)
    return bits, vals


def _operands(case, K, rng):
    if case == "random":
        a = rng.uniform(-1, 1, (32, K))
        b = rng.uniform(-1, 1, (32, K))
    elif case == "cancel":
        # pairwise-cancelling large products plus small residues: the exact sum is tiny
        # while the running partial sums are large
        a = rng.uniform(1, 2, (32, K)) * 2.0 ** rng.integers(10, 30, (32, K))
        b = rng.uniform(1, 2, (32, K)) * 2.0 ** rng.integers(10, 30, (32, K))
        a[:, 1::2] = a[:, 0::2]
        b[:, 1::2] = -b[:, 0::2]
        a[:, 0::16] = rng.uniform(-1, 1, (32, K // 16))
        b[:, 0::16] = rng.uniform(-1, 1, (32, K // 16))
    elif case == "mixed_exp":
        a = rng.uniform(-2, 2, (32, K)) * 2.0 ** rng.integers(-60, 60, (32, K))
        b = rng.uniform(-2, 2, (32, K)) * 2.0 ** rng.integers(-60, 60, (32, K))
    elif case == "subnormal":
        # products around 2^-130..2^-120 (fp32 subnormal partial sums), some normal
        a = rng.uniform(-2, 2, (32, K)) * 2.0 ** -63
        b = rng.uniform(-2, 2, (32, K)) * 2.0 ** rng.integers(-70, -57, (32, K))
        a[:, ::5] *= 2.0 ** 40
    elif case == "same_sign":
        # long same-sign accumulation: the partial sums grow to K times a product
        a = rng.uniform(0.5, 1, (32, K))
        b = rng.uniform(0.5, 1, (32, K))
    else:
        raise ValueError(case)
    return _bf16(a), _bf16(b)


@pytest.mark.parametrize("K", [16, 128, 256, 512])
@pytest.mark.parametrize("case", ["random", "cancel", "mixed_exp", "subnormal", "same_sign"])
def test_mfma_bf16_accumulation_bound(knn, case, K):
    import torch
    rng = np.random.default_rng(zlib.crc32(f"{case}-{K}".encode()))
    (ab, av), (bb, bv) = _operands(case, K, rng)
    ctx = knn.Context(0)
    try:
        dev = "cuda:0"
        ta = torch.from_numpy(ab.view(np.int16)).to(dev).view(torch.bfloat16)
        tb = torch.from_numpy(bb.view(np.int16)).to(dev).view(torch.bfloat16)
        got = ctx.mfma_probe_bf16(ta, tb).cpu().numpy().astype(np.float64)
    finally:
        ctx.close()
    worst = 0.0
    for i in range(32):
        for j in range(32):
            p = av[i] * bv[j]                       # exact in float64
            exact = math.fsum(p)
            mag = math.fsum(np.abs(p))
            err = abs(got[i, j] - exact)
            bound = 2 * U * K * mag + K * 2.0 ** -126
            assert err <= bound, (case, K, i, j, got[i, j], exact, err, bound)
            if mag > 0:
                worst = max(worst, err / (U * mag))
    # report how much of the assumed 2uK the hardware used (DESIGN.md "Certificate")
    print(f"[mfma bound] case={case} K={K}: max |err| / (u sum|p|) = {worst:.3f} (assumed <= {2 * K})")


@pytest.mark.parametrize("case", ["near_ties", "wide_range", "subnormal", "large"])
def test_bf16_data_gemm_stress(knn, oracle, case):
    """bf16 data through KNN_ALGO_GEMM (the bf16 MFMA filter with coef = (6d+32) u): inputs
    where distances differ only in their last bits, span a huge range, are subnormal or
    huge.  Results must equal the oracle on the exactly widened values."""
    rng = np.random.default_rng({"near_ties": 41, "wide_range": 42, "subnormal": 43, "large": 44}[case])
    nt, nq, d = 20000, 96, 128
    if case == "near_ties":
        # values 1 + m 2^-7 (consecutive bf16 numbers around 1): many exact ties
        tr = 1 + rng.integers(-8, 9, size=(nt, d)) * 2.0 ** -7
        te = 1 + rng.integers(-8, 9, size=(nq, d)) * 2.0 ** -7
    elif case == "wide_range":
        sc = 2.0 ** rng.integers(-40, 20, size=(1, d))
        tr = rng.standard_normal((nt, d)) * sc
        te = rng.standard_normal((nq, d)) * sc
    elif case == "subnormal":
        tr = rng.standard_normal((nt, d)) * 2.0 ** -130   # bf16 subnormals
        te = rng.standard_normal((nq, d)) * 2.0 ** -130
        tr[:, : d // 2] *= 2.0 ** 70
        te[:, : d // 2] *= 2.0 ** 70
    else:
        tr = rng.standard_normal((nt, d)) * 2.0 ** 55
        te = rng.standard_normal((nq, d)) * 2.0 ** 55
    (btr, ftr), (bte, fte) = _bf16(tr), _bf16(te)
    ftr, fte = ftr.astype(np.float32), fte.astype(np.float32)
    tl = rng.integers(0, 10, size=nt).astype(np.int32)
    ctx = knn.Context(0, algo="gemm")
    try:
        for k in (1, 10, 33, 100):
            bad, opred, odist, oidx = oracle.knn(ftr, tl, fte, k, 10)
            if bad:
                continue
            pred, dist, idx = ctx.predict(btr, tl, bte, k, 10, topk=True)
            st = ctx.stats()
            assert st["filter_operands"] == "bf16" and st["train_segments"] >= 1, st
            assert np.array_equal(idx, oidx), (case, k)
            assert np.array_equal(dist.view(np.uint32), odist.view(np.uint32)), (case, k)
            assert np.array_equal(pred, opred), (case, k)
    finally:
        ctx.close()
