"""One rank of tests/test_route_mp_gpu.py (a fresh process per rank): the real
engine behind the real exchange.  Rank r holds the contiguous slice r of every
window of the unsharded synthetic stream, partitions it on the GPU by the owner
key of its task's flow key (dist.owner_fields), exchanges the runs
(dist.route_exchange, gloo here: the runs travel through host memory) and
inserts what it received into its own Count-Min handle.  Then it asks a batch of
owner-routed queries (dist.routed_query, owners computed on the GPU).  The
exported state, the query keys and their answers go to <out>/r<rank>.npz."""
import os
import sys

import numpy as np

LAYOUTS = {"five": ["SrcIP", "DstIP", "SrcPort", "DstPort", "Protocol"], "dstip": ["DstIP"],
           "dport_proto": ["DstPort", "Protocol"]}


def record_keys(h: np.ndarray, fields) -> np.ndarray:
    """EncodeFlow keys of synthetic records (Ethernet II + IPv4 IHL 5 + TCP/UDP)."""
    cols = {"SrcIP": np.pad(h[:, 26:30], ((0, 0), (0, 12))), "DstIP": np.pad(h[:, 30:34], ((0, 0), (0, 12))),
            "SrcPort": h[:, 34:36], "DstPort": h[:, 36:38], "Protocol": h[:, 23:24]}
    return np.ascontiguousarray(np.concatenate([cols[f] for f in fields], axis=1))


def main():
    rank, world, port, out, n, steps = (int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4],
                                        int(sys.argv[5]), int(sys.argv[6]))
    layout = sys.argv[7] if len(sys.argv) > 7 else "five"
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from go2netspectra_amd import CountMin, SyntheticTraffic
    from go2netspectra_amd.dist import Router, owner_fields, route_exchange, routed_query
    fields = LAYOUTS[layout]
    seeds = np.array([0xA1, 0xB2, 0xC3, 0xD4], np.uint32)
    syn = SyntheticTraffic(flows=1 << 16)
    hdr = torch.empty((n, 64), dtype=torch.uint8, device="cuda:0")
    wl = torch.empty((n,), dtype=torch.int32, device="cuda:0")
    router = Router(world, 0, owner=owner_fields([fields]))
    cm = CountMin(1 << 16, 4, 1 << 20, 300, flow_fields=fields, seeds=seeds, max_flows=1 << 20)
    got = 0
    for k in range(steps):
        syn.fill(hdr, wl, first=(k * world + rank) * n)
        ih, iw = route_exchange(router, hdr, wl, world)
        got += int(iw.shape[0])
        cm.insert_headers(ih, iw)
    cm.flush()
    C, S, Fc, Fs = cm.export_state()
    # owner-routed queries: keys of this rank's last slice (flows present somewhere) + random keys
    keys = record_keys(hdr[:3000].cpu().numpy(), fields)
    rng = np.random.default_rng(7 + rank)
    qk = np.concatenate([keys, rng.integers(0, 256, (200, keys.shape[1]), dtype=np.uint8)])
    ans = routed_query(cm.query_many, qk, fields, world, router=router)
    np.savez(os.path.join(out, f"r{rank}.npz"), C=C, S=S, Fc=Fc, Fs=Fs, got=np.array([got]), qk=qk, ans=ans)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
