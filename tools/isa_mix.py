"""Static instruction mix of one kernel in a hipcc -save-temps .s file.
usage: python tools/isa_mix.py file.s mangled-name-substring [top]"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
names = [m.group(1) for m in re.finditer(r"^(_Z\S+):", s, re.M) if sys.argv[2] in m.group(1)]
name = names[0]
body = s[s.index(name + ":"):]
body = body[:body.index("s_endpgm")]
ops = collections.Counter()
for line in body.split("\n"):
    line = line.strip()
    if not line or line.startswith((".", ";", "_")) or line.endswith(":"):
        continue
    ops[line.split()[0]] += 1
print(name, "total", sum(ops.values()))
cls = collections.Counter()
for o, c in ops.items():
    k = ("mfma" if "mfma" in o else "valu" if o.startswith("v_") else "lds" if o.startswith("ds_")
         else "vmem" if o.startswith(("global_", "buffer_")) else "salu/smem" if o.startswith("s_") else o)
    cls[k] += c
print(dict(cls))
for o, c in ops.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 40):
    print(f"{c:6d} {o}")
