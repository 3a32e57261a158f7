"""Decodes captured in a HIP graph (pl_decode_ws, the decode on a
caller-owned workspace, exists so that a decode can be captured): the graph
replays bit-exactly against the reference's fixtures, and again after new frames
are copied into the captured input buffer -- the tree kernel (SCL L=8, SC), the
lane kernel (L=64) and LDPC BP (iteration counts too).  Every launch inside
(the frame-group counter and NaN-mask resets, the list kernel, the NaN redo
pass) is replayed from the capture."""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu


def _capture(fn):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()  # warm-up outside the capture
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    return g


def _mismatch(a, b):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape, (a.shape, b.shape)
    return int((a != b).any(axis=1).sum())


@pytest.mark.parametrize("case", ["scl8_tree", "sc_tree", "scl64_lane"])
def test_polar_decode_replayed_from_graph(gpu, case):
    from polarcode_and_ldpc_amd import _native
    if case == "scl8_tree":
        d = golden("polar_scl_1024_l8.npz")
        llr_all, exp, frozen, N, K, L = d["llr"], d["scl"], d["frozen"], 1024, 512, 8
    elif case == "sc_tree":
        d = golden("polar_p1.npz")
        llr_all, exp, frozen, N, K, L = d["llr"], d["sc"], d["frozen"], 256, 128, 0
    else:
        d = golden("polar_scl_l64.npz")
        llr_all, exp, frozen, N, K, L = d["N256_llr"], d["N256_scl"], d["N256_frozen"], 256, 128, 64
    mask = np.zeros(N, np.uint8)
    mask[frozen] = 1
    plan = _native.polar_plan(N, K, mask, L)
    h = llr_all.shape[0] // 2
    llr = torch.from_numpy(np.ascontiguousarray(llr_all[:h])).cuda()
    out = torch.empty((h, K), dtype=torch.uint8, device="cuda")
    ws = torch.empty(plan.workspace_bytes(h), dtype=torch.uint8, device="cuda")
    g = _capture(lambda: plan.decode(llr, out, ws=ws))
    for part in (slice(0, h), slice(h, 2 * h)):
        llr.copy_(torch.from_numpy(np.ascontiguousarray(llr_all[part])))
        out.fill_(7)
        g.replay()
        torch.cuda.synchronize()
        assert _mismatch(out.cpu().numpy(), exp[part]) == 0, (case, part)


def test_ldpc_decode_replayed_from_graph(gpu):
    from polarcode_and_ldpc_amd import _native
    d = golden("ldpc_bp_504.npz")
    plan = _native.ldpc_plan(d["row_ptr"], d["col_idx"], int(d["n"]), _native.PL_LDPC_BP, 20, True)
    llr_all, bits_exp, its_exp = d["zero_llr"], d["zero_bits"], d["zero_iters"]
    h = llr_all.shape[0] // 2
    llr = torch.from_numpy(np.ascontiguousarray(llr_all[:h])).cuda()
    out = torch.empty((h, int(d["n"])), dtype=torch.uint8, device="cuda")
    its = torch.empty((h,), dtype=torch.int32, device="cuda")
    ws = torch.empty(max(1, plan.workspace_bytes(h)), dtype=torch.uint8, device="cuda")
    g = _capture(lambda: plan.decode(llr, out, its, ws=ws))
    for part in (slice(0, h), slice(h, 2 * h)):
        llr.copy_(torch.from_numpy(np.ascontiguousarray(llr_all[part])))
        out.fill_(7)
        its.fill_(-1)
        g.replay()
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), bits_exp[part])
        assert np.array_equal(its.cpu().numpy(), its_exp[part])
