"""configs[3] with real processes: two fresh processes share the one GPU, each
running the real engine behind dist.route_exchange (gloo), and each shard's
state equals the sequential oracle fed the stable filter of the unsharded
stream (count_min.go:94-157 on the shard's sub-stream).  The
owner key follows the task's flow key: [SrcIP] for the 5-tuple task, the
whole key for ["DstIP"] and ["DstPort", "Protocol"] (no SrcIP: "use the full
key when SrcIP is not in the key").  Every owner-routed query must equal the
answer of the shard holding the flow (count_min.go:160-174 on that shard)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from _route_worker import LAYOUTS, record_keys  # noqa: E402


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("layout", ["five", "dstip", "dport_proto"])
def test_two_processes_route_exchange_real_engine(gpu, oracle, tmp_path, layout):
    from go2netspectra_amd import SyntheticTraffic
    from go2netspectra_amd.dist import owner_fields, owner_of_keys, owner_of_tuples
    world, n, steps = 2, 600_000, 2
    fields = LAYOUTS[layout]
    port = str(_free_port())
    worker = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_route_worker.py")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, worker, str(r), str(world), port, str(tmp_path), str(n), str(steps),
                               layout], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
             for r in range(world)]
    for p in procs:
        out, _ = p.communicate(timeout=180)
        assert p.returncode == 0, out.decode(errors="replace")[-3000:]
    # the unsharded stream of those windows, and its stable filters under the owner key
    gh, gw = SyntheticTraffic(flows=1 << 16).generate(world * steps * n)
    gh, gw = gh.cpu().numpy(), gw.cpu().numpy().view(np.uint32)
    owner = owner_fields([fields])
    tup = {f: record_keys(gh, [f]) for f in LAYOUTS["five"]}
    own = owner_of_tuples(tup["SrcIP"], tup["DstIP"], tup["SrcPort"].view(">u2").reshape(-1),
                          tup["DstPort"].view(">u2").reshape(-1), tup["Protocol"].reshape(-1), world, owner)
    K = record_keys(gh[:1], fields).shape[1]
    seeds = np.array([0xA1, 0xB2, 0xC3, 0xD4], np.uint32)
    shards = []
    for r in range(world):
        z = np.load(os.path.join(tmp_path, f"r{r}.npz"))
        m = own == r
        assert int(z["got"][0]) == int(m.sum())
        orc = oracle.CountMin(1 << 16, 4, 1 << 20, 300, K, seeds)
        assert orc.insert_hdr64(gh[m], gw[m], fields) == int(m.sum())
        oC, oS, oFc, oFs = orc.export()
        for name, a, b in (("C", z["C"], oC), ("S", z["S"], oS), ("FPc", z["Fc"], oFc), ("FPs", z["Fs"], oFs)):
            assert np.array_equal(a, b), f"rank {r}: {name}"
        shards.append(orc)
    hits = 0
    for r in range(world):
        z = np.load(os.path.join(tmp_path, f"r{r}.npz"))
        qo = owner_of_keys(z["qk"], fields, world, owner)
        want = np.array([shards[o].query(bytes(k)) for o, k in zip(qo, z["qk"])], np.uint64)
        assert np.array_equal(z["ans"], want), f"rank {r}: routed queries"
        hits += int((want != 0).sum())
    assert hits > 1000
