"""Round 5: 262 144 distinct baseline.thrift Nesting records (8 seeds x 32 768) into tmpdata/, for
NEST_FILE=tmpdata/nest_distinct_262144.bin python scripts/nested_time.py 262144 (no record repeats, unlike the
k=4096 tiled batch). tmpdata/ is not committed; delete it after the GPU run (every gpurun call sends the tree)."""
import os
import sys
from multiprocessing import Pool
sys.path.insert(0, '/root/repo')
from kitex_amd import idl, synth
def gen(seed):
    doc = idl.parse_idl('/root/repo/tests/golden/idl/baseline.thrift')
    sch = idl.to_schema(doc.struct('Nesting'))
    return b''.join(synth.thrift_records(sch, 32768, seed=seed))
os.makedirs('/root/repo/tmpdata', exist_ok=True)
with Pool(8) as p:
    parts = p.map(gen, range(100, 108))
open('/root/repo/tmpdata/nest_distinct_262144.bin', 'wb').write(b''.join(parts))
