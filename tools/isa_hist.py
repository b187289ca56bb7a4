#!/usr/bin/env python3
"""Static instruction histogram of one kernel in lib/isa/rt_kernel.s (make isa).
usage: isa_hist.py <substring of the kernel symbol> [top]"""
import collections
import re
import sys

s = open(sys.argv[2] if len(sys.argv) > 3 else "ray_tracer_fragment_shader_amd/lib/isa/rt_kernel.s").read() \
    if False else open("ray_tracer_fragment_shader_amd/lib/isa/rt_kernel.s").read()
pat = sys.argv[1]
m = re.search(r"^(_Z\S*" + re.escape(pat) + r"\S*):", s, flags=re.M)
i = m.start()
j = s.find(".Lfunc_end", i)
body = s[i:j]
ins = [l.strip() for l in body.splitlines()
       if l.strip() and not l.strip().startswith((".", ";", "//")) and not l.strip().endswith(":")]
c = collections.Counter(l.split()[0] for l in ins)
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
print(m.group(1)[:100], "instructions:", len(ins))
for k, v in c.most_common(top):
    print(f"{v:6d} {k}")
for key in ("writelane", "readlane", "s_load", "scratch", "buffer_", "s_waitcnt", "v_cndmask", "s_cbranch",
            "_f64"):
    print(key, sum(v for k, v in c.items() if key in k))
