"""Instruction statistics of selected kernels in a device .s file (tuning aid).
Usage: python tools/asmstat.py file.s substring"""
import re
import sys

s = open(sys.argv[1]).read()
pat = sys.argv[2]
for m in re.finditer(r'\n([_A-Za-z0-9]+):\s*; @', s):
    name = m.group(1)
    if pat not in name:
        continue
    end = s.find('.Lfunc_end', m.end())
    body = s[m.end():end]
    meta = {k: re.search(r'\.set ' + re.escape(name) + r'\.' + k + r', (\d+)', s) for k in ('num_vgpr', 'private_seg_size')}
    lds = re.search(r'\.amdhsa_kernel ' + re.escape(name) + r'[\s\S]*?group_segment_fixed_size (\d+)', s)
    ins = re.findall(r'^\s+([a-z_0-9]+)', body, re.M)
    c = lambda p: sum(1 for i in ins if re.match(p, i))
    print(name[:70], 'vgpr', meta['num_vgpr'].group(1) if meta['num_vgpr'] else '?',
          'scratch', meta['private_seg_size'].group(1) if meta['private_seg_size'] else '?',
          'lds', lds.group(1) if lds else '?', 'insts', len(ins), 'flat', c(r'flat_'), 'gstore', c(r'global_store'),
          'glds', c(r'global_load_lds'), 'bitop3', c(r'v_bitop3'), 'bfi', c(r'v_bfi'), 'perm', c(r'v_perm'),
          'ds_read', c(r'ds_read'), 'ds_write', c(r'ds_write'), 'barrier', c(r's_barrier'))
    waits = re.findall(r's_waitcnt[^\n]*', body)
    print('   waits:', sorted(set(waits))[:12])
