"""Static instruction mix of the fp32/Philox/M<=8 kernels (hipcc -S output)."""
import re, sys
from collections import Counter
s = open(sys.argv[1] if len(sys.argv) > 1 else '/tmp/k.s').read()
names = [m for m in re.findall(r'^(_ZN5pfmpe\w+):', s, re.M)]
for pat in ['k_propagate_weighIfLi1ELi8ELb1E', 'k_resampleIfLi1ELi8E']:
    nm = [n for n in names if pat in n][0]
    i = s.index(nm + ":"); j = s.index(".Lfunc_end", i); b = s[i:j]
    ins = re.findall(r'^\s+([vsdgbf][a-z0-9_]+)', b, re.M)
    c = Counter(ins)
    print(pat, "total", len(ins), "valu", sum(v for k, v in c.items() if k.startswith('v_')),
          "salu", sum(v for k, v in c.items() if k.startswith('s_')))
    print("   ", ", ".join(f"{k}:{v}" for k, v in c.most_common(40)))
