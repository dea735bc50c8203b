"""One-rank RCCL process group with the framework's options (high-priority collective stream):
checks that the options are accepted by this torch/RCCL build and that an async in-place
all-reduce on a slice of a flat buffer completes on the GPU (tests/test_xgmi_gpu.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from pyrecover_amd.parallel.dist import rccl_pg_options  # noqa: E402


def main():
    port = int(sys.argv[1])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    opts = rccl_pg_options()
    assert opts is not None and opts.is_high_priority_stream
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            pg_options=opts, device_id=dev)
    buf = torch.arange(1 << 20, device=dev, dtype=torch.float32).bfloat16()
    ref = buf.clone()
    work = dist.all_reduce(buf[4096:], op=dist.ReduceOp.SUM, async_op=True)
    work.wait()
    torch.cuda.synchronize()
    assert torch.equal(buf, ref)
    dist.barrier()
    dist.destroy_process_group()
    print("rccl ok")


if __name__ == "__main__":
    main()
