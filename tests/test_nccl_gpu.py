"""The RCCL (backend "nccl") branches of the multi-GPU path on the hardware, with the one
GPU of the test box as a world of one rank: route_exchange's device partition and
all-to-all, owner-routed queries (owners on the GPU), and both heavy-hitter exchanges
(device rows merged by the device sort, host arrays).  The 8-GPU run is the driver's;
this checks that the nccl code paths run and give the oracle's answers."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_nccl_world_of_one(gpu, oracle, tmp_path):
    from go2netspectra_amd import SyntheticTraffic
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = str(s.getsockname()[1])
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_nccl_worker.py")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.run([sys.executable, worker, str(tmp_path), port], env=env, capture_output=True, timeout=240)
    assert p.returncode == 0, (p.stdout + p.stderr).decode(errors="replace")[-3000:]
    z = np.load(os.path.join(tmp_path, "nccl.npz"))
    hdr, wl = SyntheticTraffic(flows=1 << 14).generate(400_000)
    hdr, wl = hdr.cpu().numpy(), wl.cpu().numpy().view(np.uint32)
    assert np.array_equal(z["ih"], hdr) and np.array_equal(z["iw"].view(np.uint32), wl)  # one shard: everything, in order
    fields = ["DstPort", "Protocol"]
    orc = oracle.CountMin(1 << 12, 4, 1 << 20, 100, 3, np.array([0xA1, 0xB2, 0xC3, 0xD4], np.uint32))
    assert orc.insert_hdr64(hdr, wl, fields) == len(wl)
    for a, b in zip((z["C"], z["S"], z["Fc"], z["Fs"]), orc.export()):
        assert np.array_equal(a, b)
    want = np.array([orc.query(bytes(k)) for k in z["qk"]], np.uint64)
    assert np.array_equal(z["ans"], want)
    assert np.array_equal(z["ans_dev"], want) and np.array_equal(z["dq"], want)
    fc, vc = orc.heavy_arrays("count")
    fs, vs = orc.heavy_arrays("size")
    for f, v, pre in ((fc, vc, "c"), (fs, vs, "s")):
        assert len(v) > 0
        assert np.array_equal(z["r" + pre], f) and np.array_equal(z["r" + pre + "v"], v)
        a, av = (z["ac"], z["acv"]) if pre == "c" else (z["as_"], z["asv"])
        assert np.array_equal(a, f) and np.array_equal(av, v)
