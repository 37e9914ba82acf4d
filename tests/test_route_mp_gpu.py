"""configs[3] with real processes: two fresh processes share the one GPU, each
running the real engine behind dist.route_exchange (gloo), and each shard's
state equals the sequential oracle fed the stable filter of the unsharded
stream (count_min.go:94-157 on the shard's sub-stream)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FIVE = ["SrcIP", "DstIP", "SrcPort", "DstPort", "Protocol"]


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_processes_route_exchange_real_engine(gpu, oracle, tmp_path):
    import torch
    from go2netspectra_amd import SyntheticTraffic
    from go2netspectra_amd.dist import shard_of
    world, n, steps = 2, 600_000, 2
    port = str(_free_port())
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_route_worker.py")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, worker, str(r), str(world), port, str(tmp_path), str(n), str(steps)],
                              env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT) for r in range(world)]
    for p in procs:
        out, _ = p.communicate(timeout=180)
        assert p.returncode == 0, out.decode(errors="replace")[-3000:]
    # the unsharded stream of those windows, and its stable filters
    gh, gw = SyntheticTraffic(flows=1 << 16).generate(world * steps * n)
    gh, gw = gh.cpu().numpy(), gw.cpu().numpy().view(np.uint32)
    owner = shard_of(np.pad(gh[:, 26:30], ((0, 0), (0, 12))), world)
    seeds = np.array([0xA1, 0xB2, 0xC3, 0xD4], np.uint32)
    for r in range(world):
        z = np.load(os.path.join(tmp_path, f"r{r}.npz"))
        m = owner == r
        assert int(z["got"][0]) == int(m.sum())
        orc = oracle.CountMin(1 << 16, 4, 1 << 20, 300, 37, seeds)
        assert orc.insert_hdr64(gh[m], gw[m], FIVE) == int(m.sum())
        oC, oS, oFc, oFs = orc.export()
        for name, a, b in (("C", z["C"], oC), ("S", z["S"], oS), ("FPc", z["Fc"], oFc), ("FPs", z["Fs"], oFs)):
            assert np.array_equal(a, b), f"rank {r}: {name}"
