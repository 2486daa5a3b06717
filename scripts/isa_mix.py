"""Static instruction mix + register metadata of kernels in a hipcc -S file: isa_mix.py <file.s> <pattern>..."""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
names = re.findall(r'^(_ZN5pfmpe\w+):', s, re.M)
for pat in sys.argv[2:]:
    for nm in [n for n in names if pat in n][:1]:
        i = s.index(nm + ":")
        j = s.index(".Lfunc_end", i)
        b = s[i:j]
        c = Counter(re.findall(r'^\s+([vsdgbf][a-z0-9_]+)', b, re.M))
        meta = {}
        for k in ['sgpr_count', 'vgpr_count', 'sgpr_spill_count', 'vgpr_spill_count', 'private_segment_fixed_size']:
            m = re.search(r'\.name:\s+' + re.escape(nm) + r'\b', s)
            blk = s[s.rfind('- .', 0, m.start()) - 4000:m.start() + 1500] if m else ''
            mm = re.findall(r'\.' + k + r':\s+(\S+)', blk)
            meta[k] = mm[-1] if mm else None
        print(pat, "valu", sum(v for k, v in c.items() if k.startswith('v_')),
              "salu", sum(v for k, v in c.items() if k.startswith('s_')), meta,
              "readfirstlane", c['v_readfirstlane_b32'], "writelane", c['v_writelane_b32'],
              "readlane", c['v_readlane_b32'], "mad_u64", c['v_mad_u64_u32'])
