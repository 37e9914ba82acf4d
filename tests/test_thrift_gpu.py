"""Thrift live path on the GPU: device decode of PacketInfo
message batches == the C restatement of UnmarshalPacketInfo, and the decoded
records drive Count-Min, SuperSpread and the exact aggregator bit-exactly."""
import numpy as np
import pytest

from helpers import thrift_messages

pytestmark = pytest.mark.gpu

FIVE = ["SrcIP", "DstIP", "SrcPort", "DstPort", "Protocol"]


def expected_records(out):
    n = len(out["ok"])
    rec = np.zeros((n, 64), np.uint8)
    ok = out["ok"].astype(bool)
    rec[~ok, 12:14] = [0x08, 0x06]
    rec[ok, 12:14] = [0x88, 0xB5]
    rec[ok, 14] = 1
    rec[ok, 15] = out["sver"][ok]
    rec[ok, 16:32] = out["src16"][ok]
    rec[ok, 32:48] = out["dst16"][ok]
    rec[ok, 48:50] = out["sport"][ok].astype(">u2").view(np.uint8).reshape(-1, 2)
    rec[ok, 50:52] = out["dport"][ok].astype(">u2").view(np.uint8).reshape(-1, 2)
    rec[ok, 52] = out["proto"][ok]
    rec[ok, 53] = out["dver"][ok]
    wl = np.where(ok, out["length"].astype(np.uint64) & 0xFFFFFFFF, 0).astype(np.uint32)
    ts = np.where(ok, out["ts"], 0)
    return rec, wl, ts


def decode_both(oracle, n, seed, bad_frac=0.1):
    from go2netspectra_amd.thrift import decode_messages, pack_messages
    rng = np.random.default_rng(seed)
    msgs = thrift_messages(rng, n, bad_frac=bad_frac)
    buf, offs = pack_messages(msgs)
    hb, nbad = decode_messages(buf, offs)
    out = oracle.thrift_decode(buf, offs)
    return hb, nbad, out


def test_decode_parity(gpu, oracle):
    hb, nbad, out = decode_both(oracle, 40_000, 1, bad_frac=0.15)
    rec, wl, ts = expected_records(out)
    assert nbad == int((out["ok"] == 0).sum()) > 0
    assert np.array_equal(hb.hdr.cpu().numpy(), rec)
    assert np.array_equal(hb.wirelen.cpu().numpy().view(np.uint32), wl)
    assert np.array_equal(hb.ts.cpu().numpy(), ts)


def test_records_drive_all_engines(gpu, oracle):
    import torch
    from go2netspectra_amd import CountMin, ExactTask, SuperSpread
    hb, nbad, out = decode_both(oracle, 60_000, 2)
    rec, wl, ts = expected_records(out)
    ok = out["ok"].astype(bool)
    seeds = np.array([0x1234, 0x5678, 0x9ABC], np.uint32)
    # Count-Min over the 5-tuple: task.go EncodeFlow of the decoded PacketInfo
    cm = CountMin(4096, 3, 1 << 16, 50, flow_fields=FIVE, seeds=seeds)
    cm.insert_headers(hb.hdr, hb.wirelen)
    cm.flush()
    orc = oracle.CountMin(4096, 3, 1 << 16, 50, 37, seeds)
    assert orc.insert_hdr64(rec, wl, FIVE) == int(ok.sum())
    C, S, Fc, Fs = cm.export_state()
    oC, oS, oFc, oFs = orc.export()
    assert np.array_equal(C, oC) and np.array_equal(S, oS)
    assert np.array_equal(Fc, oFc) and np.array_equal(Fs, oFs)
    assert cm.stats()["dropped"] == nbad
    # SuperSpread SrcIP -> DstIP
    ss = SuperSpread(2048, 2, 20, 64, 5, 0.5, 1.08, flow_fields=["SrcIP"], elem_fields=["DstIP"], seeds=seeds[:2],
                     hll_master=77, rng_seed=99)
    ss.insert_headers(hb.hdr, hb.wirelen)
    ss.flush()
    oss = oracle.SuperSpread(2048, 2, 20, 64, 5, 0.5, 1.08, 16, 16, seeds[:2], 77, 99)
    oss.insert_hdr64(rec, wl, ["SrcIP"], ["DstIP"])
    for a, b in zip(ss.export_state(), oss.export()):
        assert np.array_equal(np.asarray(a).view(np.uint8), np.asarray(b).view(np.uint8))
    # exact aggregator: per-IP versions from the message IP lengths
    ex = ExactTask("t", FIVE)
    ex.agg.insert_headers(hb.hdr, hb.wirelen, hb.ts)
    ex.flush()
    torch.cuda.synchronize()
    oex = oracle.Exact(FIVE)
    oex.insert_hdr64(rec, wl, ts)
    got = {f.Key: (f.StartTime, f.EndTime, f.PacketCount, f.ByteCount) for f in ex.flows()}
    assert got == oex.export()
