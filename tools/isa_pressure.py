"""VGPR pressure along one loop of a hipcc -S listing (diagnostic).

usage: python tools/isa_pressure.py file.s kernel-substring loop-label
Backward liveness over the loop body (two passes for the back edge); prints the
live-VGPR count every 25 instructions and the peak, with the instruction there.
"""
import re
import sys

REG = re.compile(r'\bv\[(\d+):(\d+)\]|\bv(\d+)\b')


def regs(s):
    out = set()
    for m in REG.finditer(s):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def split(ins):
    op, _, rest = ins.partition(' ')
    ops = [o.strip() for o in rest.split(',')]
    no_def = op.startswith(('ds_write', 'buffer_store', 'global_store', 'v_cmp', 'v_readlane',
                            'v_readfirstlane', 's_', 'ds_add', 'global_atomic', 'buffer_atomic',
                            'scratch_store'))
    if no_def or not ops or not ops[0]:
        return set(), regs(rest)
    d = regs(ops[0])
    u = regs(','.join(ops[1:]))
    if op.startswith('v_fmac') or op.startswith('v_mac'):
        u |= d
    return d, u


def main():
    s = open(sys.argv[1]).read()
    m = [x for x in re.finditer(r'^(_Z\S+):', s, re.M) if sys.argv[2] in x.group(1)][0]
    body = s[m.end():]
    body = body[:body.find('.Lfunc_end')]
    lines = body.split('\n')
    start = [i for i, l in enumerate(lines) if l.startswith(sys.argv[3] + ':')][0]
    end = [i for i, l in enumerate(lines)
           if i > start and re.search(r's_(cbranch_\w+|branch)\s+' + re.escape(sys.argv[3]) + r'\b', l)][0]
    ins = [l.strip() for l in lines[start + 1:end + 1]
           if l.strip() and not l.strip().startswith(('.', ';'))]
    du = [split(i) for i in ins]
    live = set()
    for _ in range(2):
        cnt = []
        for d, u in reversed(du):
            live = (live - d) | u
            cnt.append(len(live))
        cnt.reverse()
    peak = max(range(len(cnt)), key=lambda i: cnt[i])
    print(f'{len(ins)} instructions, peak live VGPRs {cnt[peak]} at #{peak}: {ins[peak]}')
    for i in range(0, len(ins), 25):
        print(f'{i:5d} {cnt[i]:4d}  {ins[i][:70]}')


if __name__ == '__main__':
    main()
