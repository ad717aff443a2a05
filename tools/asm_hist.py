"""Instruction histogram of one kernel in a hipcc -S listing: python tools/asm_hist.py file.s mangled-substring [top]"""
import collections
import sys

s = open(sys.argv[1]).read()
key = sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
name = next(l.split(':')[0] for l in s.splitlines() if ':' in l and key in l.split(':')[0] and l.startswith('_Z'))
i = s.index(name + ':')
body = s[i:s.index('.Lfunc_end', i)].splitlines()
c = collections.Counter()
for l in body:
    t = l.strip()
    if not t or t.startswith(('.', ';')) or t.endswith(':'):
        continue
    c[t.split()[0]] += 1
print(name, sum(c.values()), "instructions")
for k, v in c.most_common(top):
    print(f"{v:5d} {k}")
