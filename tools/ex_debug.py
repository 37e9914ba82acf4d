"""Debug helper: exact engine vs oracle on the test_tuples_parity stream; prints a few mismatches."""
import sys
import numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
from helpers import random_tuples
from oracle import oracle as O
from go2netspectra_amd import ExactTask, PacketBatch
FIVE = ["SrcIP", "DstIP", "SrcPort", "DstPort", "Protocol"]
for n, bp, mono in ((700, 65536, True), (1024, 65536, False), (2000, 65536, True), (1_500_000, 1 << 24, False), (300_000, 65536, True), (300_000, 65536, False)):
    rng = np.random.default_rng(1)
    t = random_tuples(rng, n, 20_000)
    ipver = np.where(t["v6"], 6, 4).astype(np.uint8)
    ts = np.arange(n, dtype=np.int64) if mono else rng.integers(-(1 << 40), 1 << 40, n).astype(np.int64)
    task = ExactTask("x", FIVE, batch_packets=bp)
    task.process_packets(PacketBatch(t["src16"], t["dst16"], t["sport"], t["dport"], t["proto"], t["length"], ipver, ts))
    task.flush()
    orc = O.Exact(FIVE)
    orc.insert_tuples(t["src16"], t["dst16"], t["sport"], t["dport"], t["proto"], ipver, t["length"], ts)
    want = orc.export()
    got = {f.Key: (f.StartTime, f.EndTime, f.PacketCount, f.ByteCount) for f in task.flows()}
    bad = [k for k in want if got.get(k) != want[k]]
    print(n, bp, mono, "flows", len(got), len(want), "bad", len(bad), "extra", len(set(got) - set(want)))
    for k in bad[:4]:
        print("  ", k, "got", got.get(k), "want", want[k])
