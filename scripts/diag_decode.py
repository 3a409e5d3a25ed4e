"""GPU diagnostics: decode a synthetic batch through the C-ABI and compare with the oracle, printing
where it differs (super-tile words of the failing call are dumped). Usage: diag_decode.py cfg n [mode]"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from kitex_amd import schema as S, synth
    from kitex_amd.codec import ThriftCodec, ProtobufCodec
    from oracle import oracle
    cfg, n = sys.argv[1], int(sys.argv[2])
    mode = sys.argv[3] if len(sys.argv) > 3 else "concat"
    reps = int(os.environ.get("REPS", "3"))
    sch = S.SCHEMAS[cfg]()
    pb = cfg == "pf"
    cs = synth.GENERATORS[cfg](n)
    rc, wire, offs = oracle.encode(sch, cs, pb=pb)
    cdc = ProtobufCodec(sch) if pb else ThriftCodec(sch)
    dev = torch.device("cuda", 0)
    buf = torch.from_numpy(wire).to(dev)
    o = torch.from_numpy(offs.astype(np.int64)).to(dev) if mode == "offsets" else None
    _, exp, est, _ = oracle.decode(sch, wire, n, offsets=offs if mode == "offsets" else None, pb=pb)
    for r in range(reps):
        res = cdc.Unmarshal(buf, n, offsets=o, raise_on_error=False)
        st = res.read_status()
        bad = []
        for c in range(len(res.columns.cols)):
            g = res.columns.cols[c]
            if isinstance(g, tuple):
                ok = np.array_equal(g[0].cpu().numpy().view(np.uint32)[:n + 1], exp.cols[c][0][:n + 1])
            else:
                gg = g.cpu().numpy()
                d = np.nonzero(gg[:n] != exp.cols[c][:n])[0]
                ok = d.size == 0
                if not ok:
                    bad.append((c, d[:5].tolist(), d.size))
            if not ok and not bad:
                bad.append((c, "var"))
        print(f"grid={os.environ.get('KX_GRID', '-')} rep {r}: code={st.code} rec={st.record} off={st.offset} "
              f"n={st.n_records} consumed={st.consumed}/{wire.size} diag={list(st.diag)} bad={bad[:3]}", flush=True)


if __name__ == "__main__":
    main()
