"""Generate tests/golden/pbn_batch_64.bin with the in-container google.protobuf (upb) — third-party, NOT the
reference — as an independent check of the nested proto3 restatement (include/kxcodec.h KX_STRUCT_PROTOBUF).

message PN (tests/pbn_cases.py: every proto3 scalar type, strings / bytes, packed repeated scalars, repeated
strings, nested and repeated messages, maps with scalar / string / message values, proto3 optional);
message Batch { repeated PN recs = 1; }. Values: tests.pbn_cases.Gen(seed 64), maps cut to at most one entry
so that the bytes do not depend on map iteration order. Run: python tests/golden/make_pbn_golden.py
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from tests import pbn_cases as P  # noqa: E402


def one_entry_maps(v, name):
    for _, fname, ty, label in P.MESSAGES[name]:
        if fname not in v:
            continue
        if label == "map":
            v[fname] = dict(list(v[fname].items())[:1])
            vt = ty[4:-1].split(",")[1]
            if vt in P.MESSAGES:
                for x in v[fname].values():
                    one_entry_maps(x, vt)
        elif ty in P.MESSAGES:
            for x in (v[fname] if label == "repeated" else [v[fname]]):
                one_entry_maps(x, ty)
    return v


def main(n=64):
    cls = P.upb_classes()
    g = P.Gen(n)
    out = bytearray()
    for _ in range(n):
        m = cls["PN"]()
        P.fill(cls, "PN", m, one_entry_maps(g.message("PN"), "PN"))
        body = m.SerializeToString(deterministic=True)
        out += b"\x0a" + P.uvarint(len(body)) + body      # Batch.recs (field 1, length-delimited)
    with open(os.path.join(HERE, f"pbn_batch_{n}.bin"), "wb") as fh:
        fh.write(bytes(out))
    print(len(out))


if __name__ == "__main__":
    main()
