"""One-shot peer-mapped all-reduce (ops/csrc/oneshot.hip, parallel/oneshot.py).

CPU: the epoch / double-slot protocol mirror (threads as ranks, random skew) never mixes epochs.
GPU: two processes sharing the one MI355X of the test box exchange IPC handles over gloo and
run the kernel against each other (on an 8-GPU node the same code maps peers over xGMI)."""
import os
import random
import subprocess
import sys
import textwrap
import threading
import time

import numpy as np
import pytest


def test_host_protocol_never_mixes_epochs():
    from spark_rapids_ml_nai_amd.parallel.oneshot import HostOneShot

    W, E, n = 4, 150, 37
    hs = HostOneShot(W, n)
    errors = []

    def rank(r):
        rng = random.Random(r)
        for e in range(1, E + 1):
            if rng.random() < 0.2:
                time.sleep(rng.random() * 1e-3)
            x = np.full(n, float(r + 1) * e)
            out = hs.allreduce(r, e, x)
            if not np.allclose(out, e * W * (W + 1) / 2.0):
                errors.append((r, e))

    ths = [threading.Thread(target=rank, args=(r,)) for r in range(W)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errors


_WORKER = textwrap.dedent("""
    import os, sys, datetime
    sys.path.insert(0, os.environ["REPO"])
    import torch, torch.distributed as dist
    os.environ["SRML_ONESHOT_TIMEOUT_S"] = "5"
    from spark_rapids_ml_nai_amd.parallel.comm import Communicator
    from spark_rapids_ml_nai_amd.parallel.oneshot import OneShotAllreduce
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    comm = Communicator(rank, world, torch.device("cpu"))
    os_ = OneShotAllreduce(comm, dev, max_bytes=64 * 1024)
    for it in range(40):
        n = 1 + (it * 997) % 8000
        for dt in (torch.float64, torch.float32):
            g = torch.Generator().manual_seed(1000 * it + rank)
            x = torch.randn(n, generator=g, dtype=torch.float64).to(dt)
            ref = sum(torch.randn(n, generator=torch.Generator().manual_seed(1000 * it + r), dtype=torch.float64)
                      .to(dt).double() for r in range(world))
            y = os_.allreduce(x.to(dev).clone())
            torch.cuda.synchronize()
            assert torch.allclose(y.cpu().double(), ref, rtol=1e-5, atol=1e-5), (rank, it, dt)
    os_.check()
    os_.close()
    dist.barrier()
    print("ONESHOT_OK", rank, flush=True)
""")


@pytest.mark.gpu
def test_oneshot_two_processes_one_gpu(tmp_path):
    script = tmp_path / "w.py"
    script.write_text(_WORKER)
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, REPO=repo, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29700 + os.getpid() % 200),
               WORLD_SIZE="2")
    procs = [subprocess.Popen([sys.executable, str(script)], env=dict(env, RANK=str(r)), stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True) for r in range(2)]
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=100)
        except subprocess.TimeoutExpired:
            p.kill()
            out, _ = p.communicate()
        outs.append(out)
    for r, (p, out) in enumerate(zip(procs, outs)):
        assert p.returncode == 0 and "ONESHOT_OK" in out, out[-3000:]


@pytest.mark.gpu
def test_oneshot_single_rank(gpu_device):
    import torch

    from spark_rapids_ml_nai_amd.parallel.comm import Communicator
    from spark_rapids_ml_nai_amd.parallel.oneshot import OneShotAllreduce

    os_ = OneShotAllreduce(Communicator(0, 1, gpu_device), gpu_device, max_bytes=8192)
    x = torch.arange(100, dtype=torch.float64, device=gpu_device)
    for _ in range(5):
        y = os_.allreduce(x.clone())
    torch.cuda.synchronize()
    assert torch.equal(y, x)
    os_.check()
    os_.close()
