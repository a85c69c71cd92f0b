"""Register / spill / wait summary of selected kernels in a device .s file (hipcc --cuda-device-only -S)."""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
pat = sys.argv[2] if len(sys.argv) > 2 else r'_Z5k_mat'
for m in re.finditer(r'^\s+\.name:\s+(\S+)\n', s, re.M):
    pass
for nm in re.findall(r'^(' + pat + r'\w*):', s, re.M):
    a = s.index(nm + ':'); b = s.index('.Lfunc_end', a)
    body = s[a:b]
    meta = s[b:b + 4000]
    g = lambda k: (re.search(r'; ' + k + r': (\d+)', meta) or [None, '?'])[1]
    w = Counter(x for x in re.findall(r's_waitcnt (vmcnt\(\d+\))', body))
    print(f"{nm[:60]}: vgpr {g('NumVgprs')} sgpr {g('NumSgprs')} scratch {g('ScratchSize')} occ {g('Occupancy')} "
          f"vspill {body.count('scratch_store')}/{body.count('scratch_load')} stores {body.count('global_store')} "
          f"barriers {body.count('s_barrier')} waits {dict(w)}")
