"""Generate tests/golden/pf_batch_64.bin with the in-container google.protobuf (upb) — third-party,
NOT the reference — as an independent check of the proto3 body restatement.

message PF { int64 a1..a8 = 1..8; string s9 = 9; string s10 = 10; }
message Batch { repeated PF recs = 1; }
Values: kitex_amd.synth.gen_pf(64) (splitmix64, seed 0x4B495445 ^ 4). Run: python tests/golden/make_pb_golden.py
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory  # noqa: E402

from kitex_amd.synth import gen_pf  # noqa: E402


def build_classes():
    fdp = descriptor_pb2.FileDescriptorProto(name="pf.proto", package="kx", syntax="proto3")
    pf = fdp.message_type.add(name="PF")
    F = descriptor_pb2.FieldDescriptorProto
    for i in range(1, 9):
        pf.field.add(name=f"a{i}", number=i, type=F.TYPE_INT64, label=F.LABEL_OPTIONAL)
    for i in (9, 10):
        pf.field.add(name=f"s{i}", number=i, type=F.TYPE_STRING, label=F.LABEL_OPTIONAL)
    b = fdp.message_type.add(name="Batch")
    b.field.add(name="recs", number=1, type=F.TYPE_MESSAGE, type_name=".kx.PF", label=F.LABEL_REPEATED)
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    get = message_factory.GetMessageClass
    return get(pool.FindMessageTypeByName("kx.PF")), get(pool.FindMessageTypeByName("kx.Batch"))


def main(n=64):
    PF, Batch = build_classes()
    cs = gen_pf(n)
    batch = Batch()
    for r in range(n):
        m = batch.recs.add()
        for i in range(8):
            setattr(m, f"a{i + 1}", int(cs.cols[i][r]))
        for j, f in enumerate((9, 10)):
            offs, data = cs.cols[8 + j]
            setattr(m, f"s{f}", bytes(data[offs[r]:offs[r + 1]]).decode())
    out = batch.SerializeToString(deterministic=True)
    with open(os.path.join(HERE, f"pf_batch_{n}.bin"), "wb") as fh:
        fh.write(out)
    print(len(out))


if __name__ == "__main__":
    main()
