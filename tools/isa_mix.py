"""Instruction mix per basic block of one kernel in a -save-temps .s file (diagnostic).
    python tools/isa_mix.py FILE.s KERNEL_SUBSTRING [min_block_size]"""
import collections
import re
import sys

path, want = sys.argv[1], sys.argv[2]
mn = int(sys.argv[3]) if len(sys.argv) > 3 else 20
lines = open(path).read().split('\n')
start = next(i for i, l in enumerate(lines) if re.match(r'^_Z\S*:', l) and want in l)
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith('.Lfunc_end'))
blocks, cur, name = [], [], 'entry'
for l in lines[start + 1:end]:
    s = l.strip()
    if re.match(r'^\.LBB\S*:', s):
        blocks.append((name, cur))
        name, cur = s.split(':')[0] + ' ' + (s.split(';')[1].strip() if ';' in s else ''), []
        continue
    if not s or s.startswith(('.', ';')):
        continue
    cur.append(s.split()[0])
blocks.append((name, cur))
tot = collections.Counter()
for name, ins in blocks:
    c = collections.Counter(ins)
    tot.update(c)
    if len(ins) >= mn:
        v = sum(n for k, n in c.items() if k.startswith('v_'))
        print(f'{name[:50]:50s} n={len(ins):5d} valu={v:5d}', ', '.join(f'{k}:{n}' for k, n in c.most_common(12)))
print('TOTAL', sum(tot.values()), ', '.join(f'{k}:{n}' for k, n in tot.most_common(30)))
