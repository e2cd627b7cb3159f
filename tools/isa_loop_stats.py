"""Instruction mix of one kernel's ISA (and of its largest basic-block loop) from a hipcc .s file.
usage: python tools/isa_loop_stats.py FILE.s MANGLED_KERNEL_NAME"""
import collections
import re
import sys

src, name = sys.argv[1], sys.argv[2]
lines = open(src).read().splitlines()
start = next(i for i, l in enumerate(lines) if l.startswith(name + ':'))
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith('.Lfunc_end'))
body = lines[start:end]
labels = {l.split(':')[0]: i for i, l in enumerate(body) if re.match(r'^\.LBB\w+:', l)}
# find backward branches (loops)
loops = []
for i, l in enumerate(body):
    m = re.match(r'\s+s_cbranch_\w+\s+(\.LBB\w+)|\s+s_branch\s+(\.LBB\w+)', l)
    if m:
        tgt = m.group(1) or m.group(2)
        if tgt in labels and labels[tgt] < i:
            loops.append((labels[tgt], i))


def mix(rng):
    c = collections.Counter()
    for l in body[rng[0]:rng[1] + 1]:
        t = l.strip().split()
        if not t or t[0].startswith(('.', ';')) or t[0].endswith(':'):
            continue
        op = t[0]
        if op.startswith('v_'):
            k = 'valu_f64' if '_f64' in op else 'valu'
            if op.startswith(('v_fma_f64', 'v_mul_f64', 'v_add_f64')):
                k = 'valu_f64_fma/mul/add'
        elif op.startswith(('global_load', 'buffer_load')):
            k = 'vmem_load'
        elif op.startswith(('global_store', 'buffer_store')):
            k = 'vmem_store'
        elif op.startswith('s_waitcnt'):
            k = 's_waitcnt'
        elif op.startswith('s_'):
            k = 'salu/smem'
        else:
            k = op
        c[k] += 1
    return c


print('whole kernel:', dict(mix((0, len(body) - 1))))
for lo, hi in sorted(loops, key=lambda r: r[1] - r[0], reverse=True)[:3]:
    c = mix((lo, hi))
    print(f'loop lines {lo}-{hi}: total={sum(c.values())}', dict(c))
