"""Shows the hazard tests/test_gpu_stream_order.py guards (DESIGN round-6 row 3b): each scenario run
as the product runs it now, and with the ordering taken out again (the FedOpt one-call step on a
private stream; the copy streams' wait for the compute stream skipped), printing whether the result
still equals the oracle. Run on the GPU box: python tools/stream_order_demo.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import test_gpu_stream_order as t  # noqa: E402


def run(fn):
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    try:
        fn()
        return "oracle-exact"
    except AssertionError as e:
        return f"WRONG: {str(e).splitlines()[0][:80]}"


def main():
    from fedn_amd import _abi
    _abi.load()
    out = {}
    out["fedopt_step_current_stream"] = run(t.test_fedopt_one_call_step_after_queued_work_on_its_buffers)
    private = torch.cuda.Stream()
    real = torch._C._cuda_getCurrentRawStream
    torch._C._cuda_getCurrentRawStream = lambda i: private.cuda_stream      # the round-6 first version
    try:
        out["fedopt_step_private_stream"] = run(t.test_fedopt_one_call_step_after_queued_work_on_its_buffers)
    finally:
        torch._C._cuda_getCurrentRawStream = real
    out["slot_h2d_with_wait"] = run(t.test_staging_slot_first_h2d_after_queued_work_on_its_block)
    out["multidev_with_wait"] = run(t.test_multidevice_slots_and_global_model_after_queued_work)
    out["waves_with_wait"] = run(t.test_wave_slots_first_h2d_after_queued_work)
    real_wait = torch.cuda.Stream.wait_stream
    torch.cuda.Stream.wait_stream = lambda self, other: None                # no copy-stream wait
    try:
        out["slot_h2d_without_wait"] = run(t.test_staging_slot_first_h2d_after_queued_work_on_its_block)
        out["multidev_without_wait"] = run(t.test_multidevice_slots_and_global_model_after_queued_work)
        out["waves_without_wait"] = run(t.test_wave_slots_first_h2d_after_queued_work)
    finally:
        torch.cuda.Stream.wait_stream = real_wait
    torch.cuda.synchronize()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
