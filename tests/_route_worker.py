"""One rank of tests/test_route_mp_gpu.py (a fresh process per rank): the real
engine behind the real exchange.  Rank r holds the contiguous slice r of every
window of the unsharded synthetic stream, partitions it on the GPU, exchanges
the runs (dist.route_exchange, gloo here: the runs travel through host memory)
and inserts what it received into its own Count-Min handle; the exported state
goes to <out>/r<rank>.npz."""
import os
import sys

import numpy as np


def main():
    rank, world, port, out, n, steps = (int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4],
                                        int(sys.argv[5]), int(sys.argv[6]))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from go2netspectra_amd import CountMin, SyntheticTraffic
    from go2netspectra_amd.dist import Router, route_exchange
    fields = ["SrcIP", "DstIP", "SrcPort", "DstPort", "Protocol"]
    seeds = np.array([0xA1, 0xB2, 0xC3, 0xD4], np.uint32)
    syn = SyntheticTraffic(flows=1 << 16)
    hdr = torch.empty((n, 64), dtype=torch.uint8, device="cuda:0")
    wl = torch.empty((n,), dtype=torch.int32, device="cuda:0")
    router = Router(world, 0)
    cm = CountMin(1 << 16, 4, 1 << 20, 300, flow_fields=fields, seeds=seeds, max_flows=1 << 20)
    got = 0
    for k in range(steps):
        syn.fill(hdr, wl, first=(k * world + rank) * n)
        ih, iw = route_exchange(router, hdr, wl, world)
        got += int(iw.shape[0])
        cm.insert_headers(ih, iw)
    cm.flush()
    C, S, Fc, Fs = cm.export_state()
    np.savez(os.path.join(out, f"r{rank}.npz"), C=C, S=S, Fc=Fc, Fs=Fs, got=np.array([got]))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
