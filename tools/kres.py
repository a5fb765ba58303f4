"""Print VGPR/SGPR/LDS/scratch of selected kernels in an amdgcn .s file."""
import re
import sys

s = open(sys.argv[1]).read()
pats = sys.argv[2:]
meta = s[s.index('amdhsa.kernels:'):]
for e in re.split(r'\n  - ', meta):
    m = re.search(r'\.name:\s+(\S+)', e)
    if m and (not pats or any(x in m.group(1) for x in pats)):
        f = {k: re.search(r'\.' + k + r':\s+(\d+)', e) for k in
             ['sgpr_count', 'vgpr_count', 'group_segment_fixed_size', 'private_segment_fixed_size']}
        print(m.group(1)[:60], {k: v.group(1) for k, v in f.items() if v})
