"""The kernels' guards report instead of faulting or dropping tiles silently.

* tile_at (pt_tile_queue.h): a schedule entry outside the launch's tiles ended the wave SILENTLY until
  round 5 -- tiles dropped, PT_OK returned.  It is now recorded in every build (guard 1) and the host
  returns PT_EKERNEL naming it.  PT_MI355_TEST_BAD_ENTRY=<position> overwrites that entry of every
  schedule the library builds with ~0u; the diffuse continuous-tiles launch and the v4 launch must
  both report it.
* The checked build (build/libpt_checked.so, -DPT_CHECKED=1): run the whole -m gpu suite under it with
  PT_MI355_LIB=build/libpt_checked.so; test_checked_build_is_loaded_when_asked pins that the library
  under test really is that build."""
from __future__ import annotations

import os

import pytest

from cpuperformanceraytracer_amd import _native as N

pytestmark = pytest.mark.gpu


@pytest.fixture
def bad_entry(monkeypatch):
    import cpuperformanceraytracer_amd as pt
    monkeypatch.setenv("PT_MI355_TEST_BAD_ENTRY", "7")
    yield pt
    monkeypatch.delenv("PT_MI355_TEST_BAD_ENTRY")
    pt.shutdown()


def _series(pt, v4: bool):
    import torch
    from cpuperformanceraytracer_amd.device import JobLauncher, check_device_errors
    W, H, S = 640, 360, 8           # 3600 tiles: scheduled (>= 512)
    buf = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda:0")
    launch = JobLauncher(buf, W, H, nframes=S, num_bounces=8, stream=torch.cuda.current_stream(), v4=v4)
    launch(1)                        # unscheduled: records the costs
    torch.cuda.synchronize()
    check_device_errors()            # (clean so far)
    launch(1 + S)                    # builds the schedule (with the bad entry) and runs it
    torch.cuda.synchronize()
    with pytest.raises(N.PtError) as ei:
        check_device_errors()
    assert ei.value.code == N.PT_EKERNEL
    assert "guard 1" in str(ei.value) and "schedule entry outside" in str(ei.value), str(ei.value)
    check_device_errors()            # reported once: the words were reset


def test_bad_schedule_entry_is_reported_diffuse(bad_entry):
    bad_entry.init(num_bounces=8)
    _series(bad_entry, v4=False)


def test_bad_schedule_entry_is_reported_v4(bad_entry):
    from cpuperformanceraytracer_amd.config import synthetic_env
    bad_entry.init(num_bounces=8)
    bad_entry.v4_config(num_bounces=8)
    bad_entry.set_env_map(synthetic_env())
    _series(bad_entry, v4=True)


def test_checked_build_is_loaded_when_asked():
    lib = os.environ.get("PT_MI355_LIB", "")
    if "checked" not in lib:
        pytest.skip("PT_MI355_LIB does not name the checked build")
    assert N.load().pt_build_checked() == 1
