"""Resource use and instruction mix of the kernels of a `hipcc --cuda-device-only -S` listing whose name matches.

  python3 scripts/isa_kernel.py <listing.s> <name substring> [...]"""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
for pat in sys.argv[2:]:
    for m in re.finditer(r'^(_ZN5pfmpe\w+):', s, re.M):
        name = m.group(1)
        if pat not in name:
            continue
        i = m.end()
        j = s.index('.Lfunc_end', i)
        body = s[i:j]
        tail = s[j:j + 3000]

        def g(key):
            r = re.search(r'; ' + key + r':\s+(\d+)', tail)
            return int(r.group(1)) if r else None
        ins = re.findall(r'^\s+([vs]_[a-z0-9_]+)', body, re.M)
        nscr = len(re.findall(r'scratch_(load|store)', body))
        c = Counter(ins)
        print(f"{name[:70]}\n  vgpr {g('NumVgprs')} sgpr {g('TotalNumSgprs')} scratch {g('ScratchSize')} "
              f"occupancy {g('Occupancy')}  static instrs {len(ins)}: valu {sum(v for k, v in c.items() if k.startswith('v_'))}"
              f" salu {sum(v for k, v in c.items() if k.startswith('s_'))} v_readlane {c['v_readlane_b32']} "
              f"v_writelane {c['v_writelane_b32']} scratch ops {nscr}")
