"""CRC32C payload-validator cases (kx_crc32c_batch / kx_frame_crc32c_validate), shared by the CPU oracle
tests and the GPU suite. Reference: crcPayloadValidator (pkg/remote/codec/validate.go:168-217), its tests
(validate_test.go:147-178: 1024-byte payload of i & 0xff; Validate(value) passes, value + "0" fails, ""
passes) and TestDefaultCodecWithCRC32_Encode_Decode (default_codec_test.go:269-316: a TTHeaderFramed frame
whose last 9 bytes are overwritten fails validation). Test infrastructure only."""
import numpy as np

from tests import frame_cases as FC

# published CRC-32C check values (RFC 3720 appendix B.4; the "123456789" catalogue check value)
KNOWN = [
    (b"123456789", 0xE3069283),
    (bytes(32), 0x8A9136AA),
    (b"\xff" * 32, 0x62A8AB43),
    (bytes(range(32)), 0x46DD794E),
    (bytes(range(31, -1, -1)), 0x113FDB5C),
    (bytes.fromhex("01c00000000000000000000000000000140000000000040000000014000000182800000000000000"
                   "0200000000000000"), 0xD9963A56),
    (b"", 0x0),
]


def py_crc32c(data: bytes) -> int:
    """independent table-driven restatement (checks the oracle's bitwise one)"""
    tab = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ 0x82F63B78 if c & 1 else c >> 1
        tab.append(c)
    c = 0xFFFFFFFF
    for b in data:
        c = tab[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def ref_payload() -> bytes:
    """validate_test.go preparePayload(): 1024 bytes, payload[i] = byte(i)"""
    return bytes(i & 0xFF for i in range(1024))


def ragged_ranges(seed: int, n: int, big: bool = True, maxlen: int = 600):
    """a buffer and n+1 offsets over it: empty ranges, 1..15 bytes, thresholds 2048 / 4096 +- 1, and
    (big) a few ranges of 100 KiB .. 1.3 MiB, all at unaligned starts. maxlen <= 190: most waves' 64
    consecutive ranges fit the kernel's 12 KiB LDS stage (kx_crc.hip), the rest read global memory"""
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, maxlen, size=n)
    special = [0, 0, 1, 7, 15, 16, 17, 2047, 2048, 2049, 4095, 4096, 4097, 8191, 8193, 64 * 4096 + 3]
    if big:
        special += [100_000, 1_300_001]
    for k, v in enumerate(special):
        if k * 7 + 3 < n:
            lens[k * 7 + 3] = v
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[0] = int(rng.integers(0, 16))  # unaligned first start
    offs[1:] = offs[0] + np.cumsum(lens).astype(np.uint64)
    data = rng.integers(0, 256, size=int(offs[n]) + 16, dtype=np.uint8)
    return data, offs


def crc_hex(v: int) -> bytes:
    return b"%08x" % v


def crc_frame(payload_msg: bytes, i: int, mode: str) -> bytes:
    """a TTHeader frame (Framed payload on odd i) carrying a "crc32c" string-KV header per mode:
    ok, bad (off by one bit), empty, upper (upper-case hex), short (7 chars), absent, extra (value + "0"),
    dup (a wrong value first, the right one last: the last assignment wins)"""
    body = FC.framed(payload_msg) if i % 2 else payload_msg
    crc = py_crc32c(body)
    kv = [(b"k%d" % (i % 3), b"v")]
    if mode == "ok":
        kv.append((b"crc32c", crc_hex(crc)))
    elif mode == "bad":
        kv.append((b"crc32c", crc_hex(crc ^ 0x10)))
    elif mode == "empty":
        kv.append((b"crc32c", b""))
    elif mode == "upper":
        kv.append((b"crc32c", crc_hex(crc).upper()))
    elif mode == "short":
        kv.append((b"crc32c", crc_hex(crc)[:7]))
    elif mode == "extra":
        kv.append((b"crc32c", crc_hex(crc) + b"0"))
    elif mode == "dup":
        kv = [(b"crc32c", crc_hex(crc ^ 1))] + kv + [(b"crc32c", crc_hex(crc))]
    return FC.ttheader(body, seqid=i, flags=1 if i % 2 else 0, int_kv=[(1, b"svc")], str_kv=kv,
                       acl=b"t" if i % 5 == 0 else None)


MODES_PASS = ("ok", "empty", "absent", "dup")
MODES_FAIL = ("bad", "upper", "short", "extra")


def crc_batch(n: int, modes, other_kinds=("framed", "mesh"), seed: int = 3):
    """n frames: TTHeader frames with crc headers cycling over `modes`, every 4th frame another framing
    (never validated). Returns schema, record bodies, frame bytes, wire, frame offsets, expected codes."""
    sch, recs = FC.records(n, start=seed)
    frames, exp = [], []
    for i in range(n):
        if other_kinds and i % 4 == 3:
            frames.append(FC.make_frame(other_kinds[i % len(other_kinds)], i, recs[i]))
            exp.append(0)
            continue
        mode = modes[(i - i // 4) % len(modes)]  # every mode occurs, framings interleaved
        msg = FC.thrift_message(b"Method%d" % (i % 7), i, recs[i])
        frames.append(crc_frame(msg, i, mode))
        body = FC.framed(msg) if i % 2 else msg
        digits_only = crc_hex(py_crc32c(body)).isdigit()  # upper-casing changes nothing: it passes
        exp.append(11 if mode in MODES_FAIL and not (mode == "upper" and digits_only) else 0)
    wire = np.frombuffer(b"".join(frames), dtype=np.uint8).copy()
    fo = np.zeros(n + 1, dtype=np.uint64)
    fo[1:] = np.cumsum([len(f) for f in frames])
    return sch, recs, frames, wire, fo, np.array(exp, dtype=np.uint8)
