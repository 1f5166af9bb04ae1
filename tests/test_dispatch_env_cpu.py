"""The hoisted step's early fork needs kernels of two queues to run side by side (a side-queue
kernel waits on the device for the main queue's TD kernel).  Environments that serialise kernel
dispatch must turn it off (engine/learner_engine.py _dispatch_serialized)."""
import pytest

from pytorch_r2d2_amd.engine.learner_engine import _dispatch_serialized


@pytest.mark.parametrize("env,want", [({}, False), ({"ROCPROF_COUNTER_COLLECTION": "1"}, True),
                                      ({"ROCPROF_COUNTER_COLLECTION": "0"}, False),
                                      ({"ROCPROF_ADVANCED_THREAD_TRACE": "1"}, True),
                                      ({"AMD_SERIALIZE_KERNEL": "3"}, True),
                                      ({"HIP_LAUNCH_BLOCKING": "1"}, True)])
def test_serialised_dispatch_detected(monkeypatch, env, want):
    for k in ("ROCPROF_COUNTER_COLLECTION", "ROCPROF_ADVANCED_THREAD_TRACE", "AMD_SERIALIZE_KERNEL",
              "HIP_LAUNCH_BLOCKING"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    assert _dispatch_serialized() is want
