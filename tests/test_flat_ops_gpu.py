"""Numerics of the flat-buffer and compression HIP kernels vs PyTorch fp32."""
import numpy as np
import pytest
import torch

from fedmi import native

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nat(gpu_device):
    return native.require()


def S():
    return native.stream_handle()


@pytest.mark.parametrize("n", [1, 7, 4096, 100003])
def test_sgd_flat(nat, gpu_device, n):
    torch.manual_seed(n)
    p = torch.randn(n, device=gpu_device)
    g = torch.randn(n, device=gpu_device)
    b = torch.randn(n, device=gpu_device)
    pr, br = p.clone(), b.clone()
    nat.sgd_flat(S(), p.data_ptr(), g.data_ptr(), b.data_ptr(), n, 0.1, 0.9, 5e-4, 0.0, False, False)
    d = g + 5e-4 * pr
    br = 0.9 * br + d
    pr = pr - 0.1 * br
    torch.cuda.synchronize()
    assert torch.allclose(b, br, rtol=1e-6, atol=1e-6)
    assert torch.allclose(p, pr, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("n,k,ties", [(62006, 620, False), (5000, 1, False), (5000, 5000, False),
                                       (1 << 20, 10000, False), (11173962, 111740, False), (70001, 700, True),
                                       (4099, 17, True), (1 << 21, 5000, "sparse")])
def test_topk_ef_exact(nat, gpu_device, n, k, ties):
    """Fused error-feedback top-k: d = x - g + r built in r, exactly the k largest |d| selected (ties:
    smallest indices), r keeps the rest; called twice on the same state (it must leave it reusable)."""
    torch.manual_seed(k)
    for rep in range(2):
        x = torch.randn(n, device=gpu_device)
        g = torch.randn(n, device=gpu_device) * 0.5
        r = torch.randn(n, device=gpu_device) * 0.1
        if ties == "sparse":                  # 100 nonzeros, k = 5000: the rest are ties at 0 (huge candidate lists)
            x.zero_(); g.zero_(); r.zero_()
            x[torch.randperm(n, device=gpu_device)[:100]] = torch.randn(100, device=gpu_device)
        elif ties:                            # many exact ties at the threshold magnitude
            x[::3] = 0.75
            g[::3] = 0.0
            r[::3] = 0.0
            x[1::7] = -0.75
            g[1::7] = 0.0
            r[1::7] = 0.0
        x[::97] = 0.0
        g[::97] = 0.0
        r[::97] = 0.0
        d = x - g + r
        if rep == 0:
            state = torch.zeros(nat.topk_state_bytes(), dtype=torch.uint8, device=gpu_device)
            cidx = torch.empty(2 * n, dtype=torch.int32, device=gpu_device)
            ckey = torch.empty(2 * n, dtype=torch.int32, device=gpu_device)
        idx = torch.full((k,), -1, dtype=torch.int32, device=gpu_device)
        val = torch.zeros(k, device=gpu_device)
        nat.topk_ef(S(), x.data_ptr(), g.data_ptr(), r.data_ptr(), n, k, state.data_ptr(), cidx.data_ptr(),
                    ckey.data_ptr(), idx.data_ptr(), val.data_ptr())
        torch.cuda.synchronize()
        assert int(idx.min()) >= 0
        sel = idx.long()
        assert len(set(sel.tolist())) == k
        assert torch.equal(d[sel], val)
        ref = d.abs().topk(k).values
        assert torch.equal(val.abs().sort(descending=True).values, ref)
        thr = ref[-1]
        tied = (d.abs() == thr).nonzero().flatten()
        chosen_tied = sel[d[sel].abs() == thr].sort().values
        assert torch.equal(chosen_tied, tied[: chosen_tied.numel()])     # smallest indices win ties
        mask = torch.ones(n, dtype=torch.bool, device=gpu_device)
        mask[sel] = False
        assert torch.equal(r[mask], d[mask])
        assert r[~mask].abs().sum().item() == 0
        off = nat.topk_overflow_offset()
        assert int(state[off:off + 4].view(torch.int32).item()) == 0      # no select ever exceeded k


def test_scatter_add_ranked_is_rank_ordered(nat, gpu_device):
    """Two ranks' top-k payloads (unique indices within a rank, overlapping across ranks) are
    applied in rank order without atomics: the result equals the sequential fp32 sum."""
    n, m = 1000, 4
    base = torch.randn(n, device=gpu_device)
    out = base.clone()
    idx = torch.tensor([[1, 5, 7, 999], [5, 2, 999, 0]], dtype=torch.int32, device=gpu_device)
    val = torch.randn(2, m, device=gpu_device)
    nat.scatter_add_ranked(S(), out.data_ptr(), idx.data_ptr(), val.data_ptr(), 2, m, 0.5, n)
    torch.cuda.synchronize()
    exp = base.clone().cpu()
    for r in range(2):
        for i in range(m):
            exp[int(idx[r, i])] += 0.5 * float(val[r, i])
    assert torch.equal(out.cpu(), exp)


def test_int8_roundtrip(nat, gpu_device):
    n = 62006
    torch.manual_seed(1)
    d = torch.randn(n, device=gpu_device)
    nch = (n + 255) // 256
    q = torch.empty(n, dtype=torch.int8, device=gpu_device)
    sc = torch.empty(nch, device=gpu_device)
    res = torch.empty(n, device=gpu_device)
    nat.quant_int8(S(), d.data_ptr(), n, q.data_ptr(), sc.data_ptr(), res.data_ptr())
    out = torch.zeros(n, device=gpu_device)
    nat.dequant_accum(S(), q.data_ptr(), sc.data_ptr(), 1, n, out.data_ptr(), 1.0)
    torch.cuda.synchronize()
    # reference quantizer
    pad = torch.zeros(nch * 256, device=gpu_device)
    pad[:n] = d
    amax = pad.view(nch, 256).abs().amax(1)
    s_ref = torch.where(amax > 0, amax / 127, torch.ones_like(amax))
    assert torch.allclose(sc, s_ref)
    deq = (torch.round(pad.view(nch, 256) / s_ref[:, None]).clamp(-127, 127) * s_ref[:, None]).view(-1)[:n]
    assert torch.allclose(out, deq, atol=1e-6)
    assert torch.allclose(res, d - deq, atol=1e-6)


def test_topk_ef_state_alternates_paths(nat, gpu_device):
    """One state reused across calls that alternate between the 2-level (< 1 M entries) and 3-level paths
    and between histogram parities: every call still selects exactly the top k."""
    torch.manual_seed(3)
    state = torch.zeros(nat.topk_state_bytes(), dtype=torch.uint8, device=gpu_device)
    for n, k in ((1 << 21, 20000), (70001, 700), (300000, 3000), (1 << 21, 9000), (62006, 620)):
        x = torch.randn(n, device=gpu_device)
        g = torch.zeros(n, device=gpu_device)
        r = torch.zeros(n, device=gpu_device)
        cidx = torch.empty(2 * n, dtype=torch.int32, device=gpu_device)
        ckey = torch.empty(2 * n, dtype=torch.int32, device=gpu_device)
        idx = torch.full((k,), -1, dtype=torch.int32, device=gpu_device)
        val = torch.zeros(k, device=gpu_device)
        nat.topk_ef(S(), x.data_ptr(), g.data_ptr(), r.data_ptr(), n, k, state.data_ptr(), cidx.data_ptr(),
                    ckey.data_ptr(), idx.data_ptr(), val.data_ptr())
        torch.cuda.synchronize()
        assert int(idx.min()) >= 0 and len(set(idx.tolist())) == k, n
        assert torch.equal(val.abs().sort(descending=True).values, x.abs().topk(k).values), n
