"""One RCCL rank (world size 1 on the test box's single GPU) for tests/test_nccl_gpu.py:
the nccl branches of the multi-GPU path run on the hardware -- route_exchange (device
partition + all-to-all), owner-routed queries, the device-resident heavy-hitter
exchange (allgather_heavy_rows) and the host-array one -- and their results go to
<out>/nccl.npz for the test to compare with the oracle."""
import os
import sys

import numpy as np


def main():
    out, port = sys.argv[1], sys.argv[2]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl"
    from go2netspectra_amd import CountMin, SyntheticTraffic
    from go2netspectra_amd.dist import (Router, allgather_heavy_arrays, allgather_heavy_rows, owner_fields,
                                        route_exchange, routed_query)
    fields = ["DstPort", "Protocol"]
    seeds = np.array([0xA1, 0xB2, 0xC3, 0xD4], np.uint32)
    hdr, wl = SyntheticTraffic(flows=1 << 14).generate(400_000)
    router = Router(1, 0, owner=owner_fields([fields]))
    ih, iw = route_exchange(router, hdr, wl, 1)
    cm = CountMin(1 << 12, 4, 1 << 20, 100, flow_fields=fields, seeds=seeds, max_flows=1 << 16)
    cm.insert_headers(ih, iw)
    cm.flush()
    h = hdr[:2000].cpu().numpy()
    qk = np.ascontiguousarray(np.concatenate([h[:, 36:38], h[:, 23:24]], axis=1))
    ans = routed_query(cm.query_many, qk, fields, 1, router=router)
    # device keys: owners, permutation, all-to-alls and answers stay on the GPU
    ans_dev = routed_query(cm.query_many, torch.from_numpy(qk).cuda(), fields, 1, router=router)
    assert ans_dev.is_cuda and ans_dev.dtype == torch.int64
    ans_dev = ans_dev.cpu().numpy().view(np.uint64)
    empty = routed_query(cm.query_many, torch.from_numpy(qk[:0]).cuda(), fields, 1, router=router)
    assert empty.is_cuda and empty.shape == (0,)
    dq = cm.query_many(torch.from_numpy(qk).cuda()).cpu().numpy().view(np.uint64)  # gns_cm_query_device
    rows = allgather_heavy_rows(cm, 1)
    arrs = allgather_heavy_arrays(cm.heavy_hitters_arrays(), 1)
    C, S, Fc, Fs = cm.export_state()
    np.savez(os.path.join(out, "nccl.npz"), ih=ih.cpu().numpy(), iw=iw.cpu().numpy(), C=C, S=S, Fc=Fc, Fs=Fs,
             qk=qk, ans=ans, ans_dev=ans_dev, dq=dq, rc=rows[0], rcv=rows[1], rs=rows[2], rsv=rows[3], ac=arrs[0], acv=arrs[1], as_=arrs[2],
             asv=arrs[3])
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
