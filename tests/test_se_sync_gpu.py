"""The split SE excitation's slice barrier under device contention.

At 256 frames the SE excitation of the 1152-channel blocks splits its first product over 5 channel
slices that meet at a software barrier (``k_bn.hip`` se_chain_kernel, ``tail.h`` group_sync).  The
launcher turns the split on only when the grid fits the device at once, but another stream's kernels
(the data-parallel trainer's RCCL all-reduce runs on a side stream during backward) can
hold the CUs the grid needs.  The barrier is bounded (2 s of wall clock); a group that times out
raises a device word every waiter polls AND a sticky word in the plan's pinned host memory, so:

* either the step completes with results bit-identical to an uncontended step,
* or the plan reports the failure -- ``B0Runtime.check_status()`` raises, every later call of the plan
  raises (``dfd_last_error`` explains why), and after ``clear_status()`` the plan runs again and is
  bit-identical to the uncontended step.

Silent wrong output is the one outcome this test rejects.  The contention is ``dfd_test_occupy``:
workgroups that each hold a whole CU's LDS and spin for a bounded time on another stream, leaving 2 of
the device's CUs to the step (fewer than one frame tile's 5 slices).  Reference error convention:
``app.py:2320-2321`` turns a raised error into an error dict.
"""
import ctypes
import time

import pytest
import torch
import torch.nn.functional as F

from deepfake_amd import _lib
from deepfake_amd.pretrained_detector import PretrainedBackboneDetector
from deepfake_amd.weights import deterministic_init_

pytestmark = pytest.mark.gpu

B, T, HW = 32, 8, 224  # 256 frames: nft = 16 frame tiles x 5 slices = 80 workgroups <= CUs -> split on
SEED = 41
OCCUPY_US = 4_000_000  # twice the barrier's 2 s budget


def _model(cuda):
    det = PretrainedBackboneDetector("efficientnet_b0", pretrained=False, num_classes=2, dropout_rate=0.0,
                                     compute_dtype="bf16")
    deterministic_init_(det, seed=SEED)
    return det.to(cuda).train()


def _inputs(cuda):
    g = torch.Generator().manual_seed(9)
    x = torch.randint(0, 256, (B, T, HW, HW, 3), generator=g, dtype=torch.uint8).to(cuda).permute(0, 1, 4, 2, 3)
    y = torch.tensor([(i * 5 + 2) % 2 for i in range(B)], device=cuda)
    return x, y


def _step(det, x, y):
    logits, _ = det(x)
    loss = F.cross_entropy(logits, y)
    loss.backward()
    return logits


def _result(det, logits):
    torch.cuda.synchronize()
    return logits.detach().cpu(), {n: p.grad.detach().cpu().clone() for n, p in det.named_parameters()}


def _same(a, b):
    la, ga = a
    lb, gb = b
    return torch.equal(la, lb) and all(torch.equal(ga[n], gb[n]) for n in ga)


def test_se_split_under_contention(cuda):
    lib = _lib.load()
    cus = torch.cuda.get_device_properties(cuda).multi_processor_count
    x, y = _inputs(cuda)

    ref_det = _model(cuda)
    ref = _result(ref_det, _step(ref_det, x, y))
    rt = ref_det.backbone.runtime()
    rt.check_status()  # an uncontended step never trips the barrier
    del ref_det

    det = _model(cuda)
    rt = det.backbone.runtime()
    side = torch.cuda.Stream(cuda)
    _lib.check(lib.dfd_test_occupy(ctypes.c_void_p(side.cuda_stream), cus - 2, OCCUPY_US))
    logits = None
    raised = None
    t0 = time.perf_counter()
    try:
        logits = _step(det, x, y)
        torch.cuda.synchronize()
        rt.check_status(synchronize=False)
    except _lib.DFDError as e:  # the barrier timed out: reported, not silent
        raised = str(e)
    side.synchronize()
    print(f"contended step + occupier: {time.perf_counter() - t0:.2f} s (occupier {OCCUPY_US / 1e6:.1f} s on {cus - 2} CUs)")
    if raised is None:
        got = _result(det, logits)
        assert _same(got, ref), "contended step completed but differs from the uncontended one (silent corruption)"
        print("contended step completed bit-identical")
        return
    assert "timed out" in raised
    print("contended step reported:", raised)
    # sticky: every later call of the plan refuses to run until cleared
    det.zero_grad(set_to_none=True)
    with pytest.raises(_lib.DFDError, match="timed out"):
        _step(det, x, y)
    rt.clear_status()
    rt.check_status()
    # the plan works again; a fresh model (the failed step moved BN running stats) matches the reference
    del det
    det = _model(cuda)
    got = _result(det, _step(det, x, y))
    det.backbone.runtime().check_status()
    assert _same(got, ref)


@pytest.mark.parametrize("expected_extra", [0, 1])
def test_group_sync_gives_up_loudly(cuda, expected_extra):
    """The barrier itself (``dfd_test_group_sync``): a group that can complete (expected = the grid)
    passes in every workgroup and raises nothing; one that never can (expected = grid + 1) makes every
    workgroup give up within the budget -- the first to time out raises the device word the others
    poll, and the host word the plans check -- instead of hanging or returning as if synchronised."""
    lib = _lib.load()
    wgs, seconds = 64, 0.5
    scratch = torch.zeros(3 + wgs, dtype=torch.int32, device=cuda)
    host = torch.zeros(1, dtype=torch.int32).pin_memory()
    stream = torch.cuda.current_stream(cuda)
    t0 = time.perf_counter()
    _lib.check(lib.dfd_test_group_sync(ctypes.c_void_p(stream.cuda_stream), wgs, wgs + expected_extra,
                                       ctypes.c_double(seconds), ctypes.c_void_p(scratch.data_ptr()),
                                       ctypes.c_void_p(host.data_ptr())))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    res = scratch[3:].cpu()
    if expected_extra == 0:
        assert torch.equal(res, torch.ones(wgs, dtype=torch.int32)), res
        assert int(host[0]) == 0 and int(scratch[2]) == 0
        assert int(scratch[0]) == 0 and int(scratch[1]) == 0  # counters back to zero at rest
    else:
        assert torch.equal(res, torch.full((wgs,), 2, dtype=torch.int32)), res
        assert int(host[0]) == 1 and int(scratch[2]) == 1
        assert seconds * 0.9 <= dt <= seconds * 3 + 1.0, dt
    print(f"group_sync expected {wgs + expected_extra} of {wgs}: {dt:.3f} s, results {res.unique().tolist()}")
