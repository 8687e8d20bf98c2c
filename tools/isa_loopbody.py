"""Print the body of one loop (by back-edge label) of one kernel in a hipcc -S
listing, and its estimated code bytes by opcode (diagnostic).

usage: python tools/isa_loopbody.py file.s kernel-substring loop-label [--print]
Sizes: VOP3/VOP3P/DS/MUBUF/SMEM encodings 8 B, VOP1/VOP2/VOPC/SOP 4 B, plus a
4-byte literal where a 32-bit constant is not an inline constant.
"""
import collections
import re
import sys

INLINE = {'0', '1', '2', '4', '-1', '-2', '-4', '0.5', '-0.5', '1.0', '-1.0', '2.0', '-2.0',
          '4.0', '-4.0', '0.15915494'}


def body(path, sub, label):
    s = open(path).read()
    m = [m for m in re.finditer(r'^(_Z\S+):', s, re.M) if sub in m.group(1)][0]
    b = s[m.end():]
    b = b[:b.find('.Lfunc_end')].split('\n')
    start = [i for i, l in enumerate(b) if l.startswith(label + ':')][0]
    end = [i for i, l in enumerate(b) if re.search(r's_c?branch\w*\s+' + re.escape(label) + r'\b', l)]
    end = max(end)
    return [l.strip() for l in b[start:end + 1] if l.strip() and not l.strip().startswith(('.', ';'))]


def size(l):
    op = l.split()[0]
    n = 4
    if op.startswith(('ds_', 'buffer_', 'global_', 'scratch_', 's_load', 's_buffer', 'v_pk', 'v_fma_',
                      'v_div_', 'v_lshl_add', 'v_add3', 'v_mad', 'v_cndmask_b32_e64', 'v_readlane',
                      'v_writelane', 'v_perm_')) or op.endswith('_e64'):
        n = 8
    if op in ('v_fmamk_f32', 'v_fmaak_f32'):
        return 8
    lits = [t for t in re.findall(r'(?<![\w.])(-?0x[0-9a-fA-F]+|-?\d+\.\d+(?:e[-+]\d+)?)', l.split(';')[0])]
    if any(t.lower() not in INLINE and not (t.startswith(('0x', '-0x')) and abs(int(t, 16)) <= 64)
           for t in lits):
        n += 4
    return n


def main():
    path, sub, label = sys.argv[1:4]
    lines = body(path, sub, label)
    c = collections.Counter()
    for l in lines:
        c[(l.split()[0], size(l))] += 1
    tot = sum(s * n for (o, s), n in c.items())
    print(f'{len(lines)} instructions, ~{tot} bytes')
    for (o, s), n in sorted(c.items(), key=lambda x: -x[1] * x[0][1])[:40]:
        print(f'  {o:30s} {s:2d} B x {n:5d} = {n * s:6d}')
    if '--print' in sys.argv:
        print('\n'.join(lines))


if __name__ == '__main__':
    main()
