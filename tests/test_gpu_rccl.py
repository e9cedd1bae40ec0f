"""The RCCL collective of the population sharding on the MI355X (one rank).

multitreegp_amd.distributed gathers the per-rank fitness / row blocks with one
all_gather_into_tensor of device buffers when the backend is RCCL ("nccl" on ROCm) and with
gloo's all_gather of host tensors otherwise; the gloo branch and all of the sharding logic run
in tests/test_distributed.py with two and three CPU ranks.  The single-GPU boxes cannot form a
two-rank RCCL group (RCCL refuses two ranks on one device, DESIGN.md "RCCL on the one-GPU pool"),
so this test runs the device collective itself (`all_gather_device`, the code both RCCL branches
call) in a one-rank RCCL group, in a child process so a failing RCCL init cannot leave state in
the test runner."""
import os
import socket
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu

_CHILD = textwrap.dedent("""
    import sys
    import torch
    import torch.distributed as dist
    from multitreegp_amd.distributed import all_gather_device, world

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:" + sys.argv[1], rank=0, world_size=1,
                            device_id=dev)
    assert dist.get_backend() == "nccl", dist.get_backend()
    assert world() == (0, 1)
    g = torch.Generator(device="cpu").manual_seed(5)
    fit = torch.randn(1001, generator=g).to(dev)          # a fitness block (+ status word)
    fit[-1] = 0.0
    rows = torch.randn(37, 1 + 3 * 5, generator=g).to(dev)  # a sharded_rows block
    for buf in (fit, rows):
        full = all_gather_device(buf, 1)
        torch.cuda.synchronize()
        assert full.device == dev and full.shape == (1,) + tuple(buf.shape), full.shape
        assert torch.equal(full[0].view(torch.int32), buf.view(torch.int32))
    dist.destroy_process_group()
    print("rccl one-rank all_gather_device ok")
""")


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_all_gather_device_one_rank():
    r = subprocess.run([sys.executable, "-c", _CHILD, str(_free_port())], capture_output=True, text=True,
                       timeout=180, cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "rccl one-rank all_gather_device ok" in r.stdout
