"""CPU check of the device decoder's entropy-decoding algorithm (CPU suite).

tests/dec_emu.cpp runs the product's own state machine (csrc/icx_decode.h) and
header parser serially, with the sync launches' threads in shuffled order, and
must reproduce the oracle's quantised coefficients (after DC prediction) for
every golden file — with and without restart intervals, for subsequence
lengths from 32 to 1024 bits (short subsequences force long resync chains).
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from tests.oracle_ffi import ROOT, load_decode_golden, noise, smooth

CSRC = os.path.join(ROOT, "image-compression_amd", "csrc")
BUILD = os.path.join(ROOT, "tests", "_build")


@pytest.fixture(scope="module")
def emu():
    os.makedirs(BUILD, exist_ok=True)
    # ICX_EMU_FLAGS: extra compile flags (tuning macros of icx_decode.h, e.g.
    # -DICX_DEC_CK_DIV=16) to check a variant's state machine before a GPU A/B
    flags = os.environ.get("ICX_EMU_FLAGS", "").split()
    lib = os.path.join(BUILD, "dec_emu%s.so" % ("_" + "_".join(f.strip("-").replace("=", "") for f in flags)
                                                 if flags else ""))
    srcs = [os.path.join(ROOT, "tests", "dec_emu.cpp"), os.path.join(CSRC, "icx_jpeg_parse.cpp")]
    deps = srcs + [os.path.join(CSRC, "icx_decode.h"), os.path.join(CSRC, "icx_jpeg_parse.h")]
    if not os.path.exists(lib) or os.path.getmtime(lib) < max(os.path.getmtime(f) for f in deps):
        # built under a name of this process, then renamed into place: test
        # workers running side by side (pytest -n) never load a half-written file
        tmp = "%s.%d.tmp" % (lib, os.getpid())
        subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-I", CSRC] + flags + ["-o", tmp] + srcs,
                       check=True)
        os.replace(tmp, lib)
    L = ctypes.CDLL(lib)
    L.dec_emu_coefs.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    return L


def run(emu, data, nb, seed, sub):
    buf = np.frombuffer(data, np.uint8)
    out = np.zeros((nb, 64), np.int16)
    it = ctypes.c_int()
    rc = emu.dec_emu_coefs(buf.ctypes.data, buf.size, out.ctypes.data, nb, seed, sub, ctypes.byref(it))
    return rc, out, it.value


@pytest.mark.parametrize("sub", [32, 160, 1024])
def test_emulated_sync_decode_matches_oracle(emu, oracle, sub):
    meta, jpgs, _ = load_decode_golden()
    iters = []
    for k, (name, data) in enumerate(jpgs.items()):
        if meta["cases"][name].get("unsupported"):
            continue
        ref = oracle.jpeg_coefs(data)
        rc, got, it = run(emu, data, ref.shape[0], seed=k + 1, sub=sub)
        assert rc == 0, (name, rc)
        assert np.array_equal(got, ref), name
        iters.append(it)
    if sub >= 1024:  # tiny subsequences (shorter than many codes) are a correctness stress only
        assert max(iters) <= 40, max(iters)


def test_emulated_decode_of_own_encodes(emu, oracle):
    for (h, w), q, gen in [((72, 120), 0.25, smooth), ((64, 96), 0.95, noise), ((33, 47), 1.0, noise)]:
        data = oracle.encode(gen(h, w, 7), q)
        ref = oracle.jpeg_coefs(data)
        rc, got, _ = run(emu, data, ref.shape[0], seed=3, sub=256)
        assert rc == 0 and np.array_equal(got, ref), (h, w, q)


def test_fuzzed_streams_never_read_out_of_bounds(oracle, tmp_path):
    """Corrupted files through the product parser + walker under
    AddressSanitizer: every call must end (status 0 or corrupt/unsupported)
    without an out-of-bounds access.  Guards the device kernels' indexing,
    which share this code."""
    lib = os.path.join(BUILD, "dec_emu_asan.so")
    srcs = [os.path.join(ROOT, "tests", "dec_emu.cpp"), os.path.join(CSRC, "icx_jpeg_parse.cpp")]
    exe = str(tmp_path / "fuzz")
    main = tmp_path / "fuzz_main.cpp"
    main.write_text(r'''
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <vector>
extern "C" int dec_emu_coefs(const uint8_t*, size_t, int16_t*, size_t, int, int, int*);
int main(int argc, char** argv) {
    FILE* f = fopen(argv[1], "rb");
    std::vector<uint8_t> buf(1 << 22);
    size_t n = fread(buf.data(), 1, buf.size(), f);
    fclose(f);
    std::vector<int16_t> out((size_t)64 * 200000);
    int it = 0, bad = 0;
    size_t pos = 0;
    while (pos + 4 <= n) {  // records: u32 length, bytes
        uint32_t len = buf[pos] | buf[pos + 1] << 8 | buf[pos + 2] << 16 | (uint32_t)buf[pos + 3] << 24;
        pos += 4;
        std::vector<uint8_t> one(buf.begin() + pos, buf.begin() + pos + len);  // exact-size copy: ASan sees overruns
        int rc = dec_emu_coefs(one.data(), one.size(), out.data(), 200000, 2, 256, &it);
        if (rc != 0 && rc != 4 && rc != 5 && rc != 6) bad++;
        pos += len;
    }
    printf("bad=%d\n", bad);
    return bad != 0;
}
''')
    r = subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-fsanitize=address", "-fno-omit-frame-pointer", "-I", CSRC,
                        "-o", exe, str(main)] + srcs, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    meta, jpgs, _ = load_decode_golden()
    rng = np.random.default_rng(1234)
    recs = []
    names = [k for k in jpgs if not meta["cases"][k].get("unsupported")]
    for i in range(400):
        d = bytearray(jpgs[names[i % len(names)]])
        mode = i % 4
        if mode == 0:    # flip random bytes in the entropy-coded data
            for _ in range(int(rng.integers(1, 8))):
                p = int(rng.integers(len(d) // 2, len(d)))
                d[p] = int(rng.integers(0, 256))
        elif mode == 1:  # truncate
            d = d[: int(rng.integers(4, len(d)))]
        elif mode == 2:  # insert stray markers (RSTn, fill, EOI)
            for _ in range(int(rng.integers(1, 4))):
                p = int(rng.integers(len(d) // 2, len(d)))
                d[p:p] = bytes([0xFF, int(rng.choice([0xD0, 0xD3, 0xD9, 0xFF, 0xC4]))])
        else:            # corrupt header bytes (tables, dimensions, sampling)
            for _ in range(int(rng.integers(1, 4))):
                p = int(rng.integers(2, min(len(d), 700)))
                d[p] = int(rng.integers(0, 256))
        recs.append(len(d).to_bytes(4, "little") + bytes(d))
    fz = tmp_path / "cases.bin"
    fz.write_bytes(b"".join(recs))
    r = subprocess.run([exe, str(fz)], capture_output=True, text=True, timeout=600,
                       env={**os.environ, "ASAN_OPTIONS": "detect_leaks=0"})
    assert r.returncode == 0 and "bad=0" in r.stdout, (r.stdout[-500:], r.stderr[-3000:])


@pytest.mark.parametrize("sub", [4096, 16384, 32768, 65536])  # 65536: 16 checkpoint intervals
def test_emulated_checkpoint_early_exit(emu, oracle, sub):
    """Subsequences long enough to carry sync checkpoints (dec_sync_walk):
    re-walks stop where they meet their previous walk, and the coefficients
    (block counts spliced from the checkpoints included) still match the
    oracle, with and without warm-up estimates (odd / even seeds)."""
    early = 0
    for (h, w), q, gen in [((320, 480), 0.95, noise), ((360, 640), 0.9, smooth), ((256, 256), 1.0, noise)]:
        data = oracle.encode(gen(h, w, 11), q)
        ref = oracle.jpeg_coefs(data)
        for seed in (1, 2, 5):
            rc, got, _ = run(emu, data, ref.shape[0], seed=seed, sub=sub)
            assert rc == 0 and np.array_equal(got, ref), (h, w, q, seed)
            early += ctypes.c_long.in_dll(emu, "dec_emu_early").value
    assert early > 0


def test_lean_walk_equals_full_walk(emu, oracle):
    """k_dec_init / k_dec_sync walk DecLean tables (state transitions only:
    bits consumed, zig-zag advance) while the write pass walks the full
    tables.  From random states (almost all wrong starts: invalid codes,
    runs past index 63, jumps over restart pads) both state machines must
    agree after every symbol, on the golden files (restart intervals, grey,
    4:2:2 / 4:4:4, RGB) and on q95-1.0 noise, where most symbols carry
    long extra-bit fields."""
    emu.dec_emu_lean_check.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    emu.dec_emu_lean_check.restype = ctypes.c_long
    meta, jpgs, _ = load_decode_golden()
    files = [d for n, d in jpgs.items() if not meta["cases"][n].get("unsupported")]
    files += [oracle.encode(noise(96, 128, 5), q) for q in (0.95, 1.0)] + [oracle.encode(smooth(64, 80, 2), 0.5)]
    checked = 0
    for k, data in enumerate(files):
        buf = np.frombuffer(data, np.uint8)
        bad = emu.dec_emu_lean_check(buf.ctypes.data, buf.size, 64, 400, k + 1)
        assert bad == 0, (k, bad)
        checked += 1
    assert checked > 100
    # the lean walkers step symbol pairs (icx_decode.h): each pair step was
    # checked against two of the spec's single steps
    assert ctypes.c_long.in_dll(emu, "dec_emu_pairs").value > 1000


@pytest.mark.parametrize("sub", [64, 1024, 16384])
def test_emulated_decode_flags_every_damaged_file_it_would_get_wrong(emu, oracle, sub):
    """The device's entropy decode on the recovery fixtures (truncation, bad
    codes, RSTn missing / duplicated / renumbered, bad trailers): every file
    either comes back flagged (ICX_E_CORRUPT: the host route with IJG 6b's
    recovery, icx_seqdecode.cpp) or with exactly the oracle's coefficients -
    never accepted with others.  Intact files are never flagged."""
    import json
    z = np.load(os.path.join(ROOT, "tests", "golden", "recovery_golden.npz"))
    with open(os.path.join(ROOT, "tests", "golden", "recovery_golden.json")) as f:
        meta = json.load(f)
    flagged = accepted = 0
    for k, name in enumerate(sorted(meta["cases"])):
        data = z[f"jpg:{name}"].tobytes()
        ref = oracle.jpeg_coefs(data)
        nb = len(ref) if ref is not None else 1 << 16
        rc, got, _ = run(emu, data, nb, k, sub)
        if name.endswith("_intact"):
            assert rc == 0, name
        if rc == 0:
            assert ref is not None and np.array_equal(got, ref), name
            accepted += 1
        else:
            assert rc == 6, (name, rc)
            flagged += 1
    assert flagged >= 150 and accepted >= 20


def test_emulated_decode_fuzz_never_accepts_a_wrong_decode(emu, oracle):
    """Random damage (cuts, byte flips, planted 0xFF runs, RSTn removed /
    renumbered, bytes inserted, markers planted) on small files of every
    layout: the emulated device decode is flagged or equals the oracle."""
    import io
    from PIL import Image
    rng = np.random.default_rng(606)
    flagged = accepted = 0
    for i in range(400):
        h, w = int(rng.integers(8, 70)), int(rng.integers(8, 70))
        img = smooth(h, w, i) if i % 2 else noise(h, w, i)
        kw = dict(quality=int(rng.integers(30, 100)), subsampling=int(rng.integers(0, 3)))
        if i % 3 == 0:
            kw["restart_marker_blocks"] = int(rng.integers(1, 6))
        buf = io.BytesIO()
        Image.fromarray(img if i % 5 else img[:, :, 0]).save(buf, "JPEG", **kw)
        d = bytearray(buf.getvalue())
        sos = d.index(b"\xff\xda")
        s0 = sos + 2 + int.from_bytes(d[sos + 2:sos + 4], "big")
        op = int(rng.integers(0, 6))
        if op == 0:
            d = d[:int(rng.integers(s0, len(d)))]
        elif op == 1:
            d[int(rng.integers(s0, len(d) - 2))] = int(rng.integers(0, 256))
        elif op == 2 and len(d) > s0 + 10:
            a = int(rng.integers(s0, len(d) - 8))
            d[a:a + 6] = b"\xff\x00" * 3
        elif op == 3:
            r = [k for k in range(s0, len(d) - 1) if d[k] == 0xFF and 0xD0 <= d[k + 1] <= 0xD7]
            if r:
                k = r[int(rng.integers(0, len(r)))]
                d = d[:k] + d[k + 2:] if rng.random() < 0.5 else d[:k + 1] + bytes([0xD0 + int(rng.integers(0, 8))]) + d[k + 2:]
        elif op == 4:
            a = int(rng.integers(s0, len(d) - 1))
            d = d[:a] + bytes(rng.integers(0, 256, int(rng.integers(1, 5)), dtype=np.uint8)) + d[a:]
        else:
            a = int(rng.integers(s0, len(d) - 1))
            d = d[:a] + bytes([0xFF, int(rng.choice([0xD9, 0xC4, 0xFE, 0x01, 0xD3]))]) + d[a:]
        data = bytes(d)
        ref = oracle.jpeg_coefs(data)
        nb = len(ref) if ref is not None else 1 << 16
        rc, got, _ = run(emu, data, nb, i, int(rng.choice([64, 512, 4096])))
        if rc == 0:
            assert ref is not None and np.array_equal(got, ref), (i, op, kw)
            accepted += 1
        else:
            flagged += 1
    assert accepted >= 40 and flagged >= 200
