"""RCCL on the hardware at world size 1 (the ``nccl`` branches had only
run through gloo).  One GPU cannot host two RCCL ranks (one rank per device), so the two-rank
transport stays unmeasured here; what one rank CAN check on the real library is every call the
bench and the pipeline make outside the point-to-point hand-offs: ``init_process_group("nccl",
device_id=...)`` (bench.py main), barrier, all_reduce(MAX) of a device tensor (the bench's
max-over-ranks timing), broadcast (the pipeline's NLL / token checks), ``new_group`` (the
pipeline's first <-> last stage token communicator), and a clean teardown.  Run in a child
process so the default process group never leaks into the other GPU tests."""
import os
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu

CHILD = textwrap.dedent("""
    import torch, torch.distributed as dist
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
    dist.barrier()
    t = torch.tensor([3.25, -1.0], device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ok = torch.tensor([1], device=dev, dtype=torch.int32)
    dist.broadcast(ok, src=0)
    g = dist.new_group([0])
    x = torch.arange(8, device=dev, dtype=torch.float16)
    dist.all_reduce(x, group=g)
    torch.cuda.synchronize()
    assert t.tolist() == [3.25, -1.0] and int(ok) == 1 and x.tolist() == list(range(8))
    dist.barrier()
    dist.destroy_process_group()
    print("rccl ok", torch.cuda.nccl.version() if hasattr(torch.cuda, "nccl") else "")
""")


def test_rccl_world1_collectives():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29517", RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "rccl ok" in r.stdout, r.stdout
