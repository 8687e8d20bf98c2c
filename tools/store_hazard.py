"""Scan gfx950 assembly for a VMEM store of more than 8 bytes (dwordx3 / x4)
directly followed (no wait state) by a VALU write of one of its data VGPRs.
Observed on MI355X (ROCm 7.2 hipcc emits it with no wait state): the store
read the last lanes of its data register after the VALU overwrote it."""
import re
import sys

ST = re.compile(r'^\s*(buffer|global|flat|scratch)_store_dwordx([34])\s+(.*)$')
VALU = re.compile(r'^\s*(v_\w+)\s+(v\[(\d+):(\d+)\]|v(\d+))')


def regs_of(data):
    m = re.match(r'v\[(\d+):(\d+)\]', data)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r'v(\d+)', data)
    return {int(m.group(1))} if m else set()


def scan(path):
    lines = open(path).read().split('\n')
    fn = '?'
    hits = []
    for i, l in enumerate(lines):
        if re.match(r'^_Z\w+:', l):
            fn = l.split(':')[0]
        m = ST.match(l)
        if not m:
            continue
        ops = [o.strip() for o in m.group(3).split(',')]
        data = ops[1] if m.group(1) == 'global' and ops[0].startswith('v') and len(ops) > 2 and ops[1].startswith('v[') else ops[0]
        if m.group(1) in ('buffer', 'scratch'):
            data = ops[0]
        elif m.group(1) in ('global', 'flat'):
            data = ops[1]
        dr = regs_of(data)
        n = 0
        j = i + 1
        while j < len(lines) and n < 1:
            t = lines[j].strip()
            j += 1
            if not t or t.startswith(';') or t.startswith('.') or t.endswith(':'):
                continue
            n += 1
            if t.startswith('s_nop'):
                break
            v = VALU.match(t)
            if v and not t.startswith('v_readlane') and not t.startswith('v_readfirstlane'):
                w = (set(range(int(v.group(3)), int(v.group(4)) + 1)) if v.group(3)
                     else {int(v.group(5))})
                if w & dr:
                    hits.append((fn, i + 1, l.strip(), t))
                    break
    return hits


if __name__ == '__main__':
    tot = 0
    for p in sys.argv[1:]:
        for fn, ln, a, b in scan(p):
            tot += 1
            print(f"{p}:{ln} {fn[:90]}\n    {a}\n    {b}")
    print("hazards:", tot)
