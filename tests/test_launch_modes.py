"""How a run spreads over GPUs, on CPU: bench.py's --gpus resolution (the
driver's torchrun launch, the in-process multi-device context, one GPU, and
the loud failures: --gpus larger than the visible GPUs, --gpus != WORLD_SIZE),
and the C-ABI's multi-device constructor rejecting a bad device list before
any HIP call (rtw_create_devices, include/rtw.h; SURVEY.md §8(b)(1)'s
device_mask context).  The GPU side -- a one-device context bit-identical to
rtw_render -- is tests/test_gpu_multidevice.py."""
import ctypes as C
import os
import subprocess
import sys

import pytest

import ray_tracing_weekend_amd as rtw

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_resolve_launch_modes():
    import bench
    assert bench.resolve_launch(1, {}, 0) == ("single", 1)
    assert bench.resolve_launch(1, {"WORLD_SIZE": "1"}, 8) == ("single", 1)
    assert bench.resolve_launch(8, {"WORLD_SIZE": "8"}, 8) == ("torchrun", 8)
    assert bench.resolve_launch(2, {}, 8) == ("inproc", 2)
    assert bench.resolve_launch(8, {}, 8) == ("inproc", 8)


@pytest.mark.parametrize("gpus,env,visible", [
    (2, {}, 1),                     # asks for more GPUs than the box has: never a silent n_gpus 1
    (8, {}, 0),
    (4, {"WORLD_SIZE": "8"}, 8),    # torchrun world and --gpus disagree
    (8, {"WORLD_SIZE": "2"}, 8),
    (0, {}, 8),
])
def test_resolve_launch_fails_loudly(gpus, env, visible):
    import bench
    with pytest.raises(SystemExit) as e:
        bench.resolve_launch(gpus, env, visible)
    assert e.value.code not in (0, None)


def test_bench_gpus_2_without_gpus_exits_nonzero():
    """`python bench.py --gpus 2` on a box with fewer GPUs ends with an error
    and prints no JSON line (here: no GPU at all)."""
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("two GPUs visible")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1",
                        "--warmup", "0"], capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode != 0
    assert "--gpus 2" in p.stderr and "visible" in p.stderr
    assert '"metric"' not in p.stdout


def _create(devs, prec=rtw.RTW_F64):
    arr = (C.c_int * max(len(devs), 1))(*devs)
    out = C.c_void_p(12345)
    rc = rtw._lib.rtw_create_devices(arr, len(devs), prec, C.byref(out))
    return rc, out.value


@pytest.mark.parametrize("devs", [[0, 0], [1, 0, 1], [3, 3], [-1], [0, -2]])
def test_create_devices_rejects_repeated_or_negative_devices(devs):
    rc, ctx = _create(devs)
    assert rc == rtw._capi.RTW_E_INVALID and ctx is None


def test_create_devices_rejects_empty_list_and_bad_precision():
    assert _create([]) == (rtw._capi.RTW_E_INVALID, None)
    assert _create([0], prec=7) == (rtw._capi.RTW_E_INVALID, None)
    assert rtw._lib.rtw_create_mask(0, rtw.RTW_F64) is None
    with pytest.raises(rtw.RenderError):
        rtw.Renderer(precision=rtw.RTW_F64, devices=[0, 0])


def test_create_devices_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    rc, ctx = _create([0])
    assert rc < 0 and ctx is None
    assert rtw._lib.rtw_create_mask(1, rtw.RTW_F64) is None
