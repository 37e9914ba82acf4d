"""CPU: whole-frame decode of the pcap packer (gns_frame.cpp, gns_frame_record)
against the hand-derived golden frames (tests/golden/frame_vectors.json) and
against the independent restatement oracle/pyframe.py (gopacket v1.1.19 +
parser.go:37-61), plus a mutation fuzz where the two must agree byte for byte.
gns_frame_record is host code: these tests make no GPU call."""
import ctypes as ct
import json
import os

import numpy as np
import pytest

import go2netspectra_amd as g
from go2netspectra_amd import _lib
from oracle import pyframe

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
VECTORS = json.load(open(os.path.join(GOLD, "frame_vectors.json")))["vectors"]


def c_record(frame: bytes, wirelen: int):
    L = _lib.load()
    buf = ct.create_string_buffer(bytes(frame), max(1, len(frame)))
    rec = ct.create_string_buffer(64)
    rc = L.gns_frame_record(buf, len(frame), wirelen, rec)
    assert rc in (0, 1, 2), rc
    return rc, rec.raw


def expected_tuple(e):
    if e is None:
        return None
    src, dst = bytes.fromhex(e["src"]), bytes.fromhex(e["dst"])
    return (src + bytes(16 - len(src)), dst + bytes(16 - len(dst)), e["sport"], e["dport"], e["proto"], e["ver"])


def record_tuple(rec: bytes):
    """(tuple) of a 0x88B5 record, None for the drop record"""
    if rec[12:14] == b"\x08\x06":
        return None
    assert rec[12:15] == b"\x88\xb5\x01"
    assert rec[15] == rec[53]
    return (rec[16:32], rec[32:48], int.from_bytes(rec[48:50], "big"), int.from_bytes(rec[50:52], "big"), rec[52],
            rec[15])


@pytest.mark.parametrize("v", VECTORS, ids=[v["name"] for v in VECTORS])
def test_pyframe_golden(v):
    frame = bytes.fromhex(v["frame"])
    assert pyframe.frame_tuple(frame) == expected_tuple(v["expect"]), v["note"]
    assert pyframe.fast_shape(frame, v["wirelen"]) == v["verbatim"]


@pytest.mark.parametrize("v", VECTORS, ids=[v["name"] for v in VECTORS])
def test_c_frame_record_golden(v, oracle):
    frame = bytes.fromhex(v["frame"])
    rc, rec = c_record(frame, v["wirelen"])
    want = expected_tuple(v["expect"])
    if v["verbatim"]:
        assert rc == 0 and rec == frame[:64] + bytes(max(0, 64 - len(frame)))
        # the device parser (restated by the C oracle) reads the expected tuple off the verbatim record
        st, src, dst, sp, dp, pr = oracle.parse_hdr64(rec, v["wirelen"])
        assert (st, src, dst, sp, dp, pr) == (0, want[0], want[1], want[2], want[3], want[4])
    else:
        assert rc == (2 if want is None else 1)
        assert record_tuple(rec) == want, v["note"]
        st, src, dst, sp, dp, pr = oracle.parse_hdr64(rec, v["wirelen"])
        if want is None:
            assert st == 1  # dropped: not an IP packet
        else:
            assert (st, src, dst, sp, dp, pr) == (0,) + want[:5]
    assert rec == pyframe.frame_record(frame, v["wirelen"])


def _mutants(rng, n):
    base = [(bytes.fromhex(v["frame"]), v["wirelen"]) for v in VECTORS]
    for i in range(n):
        f, wl = base[int(rng.integers(len(base)))]
        f = bytearray(f)
        kind = int(rng.integers(4))
        if kind == 0 and len(f) > 1:  # snap
            f = f[: int(rng.integers(1, len(f) + 1))]
        elif kind == 1:  # flip header bytes
            for _ in range(int(rng.integers(1, 4))):
                j = int(rng.integers(min(len(f), 90))) if f else 0
                if f:
                    f[j] = int(rng.integers(256))
        elif kind == 2:  # length fields / flags in the first 90 bytes, biased to small values
            for _ in range(int(rng.integers(1, 3))):
                if f:
                    j = int(rng.integers(min(len(f), 90)))
                    f[j] = int(rng.choice([0, 1, 2, 4, 5, 6, 8, 0x11, 0x40, 0x80, 0xFF]))
        else:  # append junk
            f += bytes(rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8))
        wl2 = max(len(f), wl) if rng.random() < 0.7 else len(f) + int(rng.integers(0, 3000))
        yield bytes(f), wl2


def test_c_matches_pyframe_fuzz():
    rng = np.random.default_rng(7)
    kinds = [0, 0, 0]
    for f, wl in _mutants(rng, 30000):
        rc, rec = c_record(f, wl)
        kinds[rc] += 1
        assert rec == pyframe.frame_record(f, wl), (f.hex(), wl)
    assert min(kinds) > 100, kinds  # every outcome exercised


def test_packer_escapes_every_golden_frame(tmp_path):
    frames = [bytes.fromhex(v["frame"]) for v in VECTORS]
    wl = [v["wirelen"] for v in VECTORS]
    path = str(tmp_path / "golden.pcap")
    g.write_pcap(path, frames, wl)
    hb = g.read_pcap(path)
    assert len(hb) == len(frames)
    for i, (f, w) in enumerate(zip(frames, wl)):
        assert bytes(hb.hdr[i]) == pyframe.frame_record(f, w), VECTORS[i]["name"]
        assert hb.wirelen[i] == w
    counts = (ct.c_uint64 * 3)()
    L = _lib.load()
    L.gns_pack_counts(counts)  # the counts of this thread's last pack
    want = [sum(v["verbatim"] for v in VECTORS), sum(not v["verbatim"] and v["expect"] is not None for v in VECTORS),
            sum(v["expect"] is None for v in VECTORS)]
    assert list(counts) == want


def _build_sanitized(tmp_path):
    """gns_frame.cpp + gns_pcap.cpp + tests/sanitize_driver.cpp, host code only, under
    AddressSanitizer and UndefinedBehaviorSanitizer (the hand-restated
    gopacket decoder is fuzzed under a sanitizer build)."""
    import shutil
    import subprocess
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    here = os.path.dirname(os.path.abspath(__file__))
    csrc = os.path.join(here, "..", "go2netspectra_amd", "csrc")
    exe = str(tmp_path / "gns_sanitize")
    cmd = [hipcc, "-x", "hip", "--cuda-host-only", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           os.path.join(csrc, "gns_frame.cpp"), os.path.join(csrc, "gns_pcap.cpp"),
           os.path.join(here, "sanitize_driver.cpp"), "-o", exe, "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return exe


def test_host_decoders_under_sanitizers(tmp_path):
    """The whole-frame decoder, the compact-record packing and the pcap/pcapng
    packers on mutated inputs, built with ASan + UBSan: no report, and every frame's
    record and compact record equal the product library's."""
    import subprocess
    exe = _build_sanitized(tmp_path)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    rng = np.random.default_rng(99)
    frames = list(_mutants(rng, 8000))
    blob = bytearray()
    for f, wl in frames:
        blob += np.array([len(f), wl], np.uint32).tobytes() + f
    fin, fout = tmp_path / "frames.bin", tmp_path / "frames.out"
    fin.write_bytes(bytes(blob))
    r = subprocess.run([exe, "frames", str(fin), str(fout)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "runtime error" not in r.stderr, r.stderr[-3000:]
    out = fout.read_bytes()
    assert len(out) == 82 * len(frames)
    for i, (f, wl) in enumerate(frames):
        o = out[82 * i: 82 * (i + 1)]
        rc, rec = c_record(f, wl)
        assert o[0] == rc and o[1:65] == rec, i
    # captures: well-formed, truncated at random points, and with flipped header bytes
    vec = [bytes.fromhex(v["frame"]) for v in VECTORS]
    wls = [v["wirelen"] for v in VECTORS]
    paths = []
    for k, writer in enumerate((g.write_pcap, g.write_pcapng)):
        base = tmp_path / f"cap{k}"
        writer(str(base), vec, wls)
        data = base.read_bytes()
        paths.append(str(base))
        for j in range(12):
            m = bytearray(data)
            if j % 2:
                m = m[: int(rng.integers(1, len(m)))]
            else:
                for _ in range(3):
                    m[int(rng.integers(len(m)))] = int(rng.integers(256))
            p = tmp_path / f"cap{k}_{j}"
            p.write_bytes(bytes(m))
            paths.append(str(p))
    r = subprocess.run([exe, "pcap"] + paths, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "runtime error" not in r.stderr, r.stderr[-3000:]
    lines = r.stdout.split("\n")
    assert lines[0].split()[0] == lines[0].split()[1] == str(len(vec))
