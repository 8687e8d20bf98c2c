"""Instruction mix of the loops of one kernel in a hipcc -S listing (diagnostic).

usage: python tools/isa_loops.py file.s [kernel-substring]
Prints, per loop (back-edge), its length and the counts of VALU / packed /
v_mov / LDS / VMEM / scalar / waitcnt / scratch instructions.
"""
import collections
import re
import sys


def kernel_body(s, sub):
    for m in re.finditer(r'^(_Z\S+):', s, re.M):
        if sub in m.group(1):
            body = s[m.end():]
            return body[:body.find('.Lfunc_end')]
    raise SystemExit(f"no kernel matching {sub}")


def mix(seg):
    c = collections.Counter()
    for l in seg:
        op = l.split()[0]
        if op.startswith('v_pk'):
            c['v_pk'] += 1
        elif op.startswith('v_mov') or op.startswith('v_accvgpr'):
            c['v_mov'] += 1
        elif op.startswith('v_'):
            c['valu'] += 1
        elif op.startswith('ds_'):
            c['ds'] += 1
        elif op.startswith(('buffer_', 'global_')):
            c['vmem'] += 1
        elif op.startswith('scratch'):
            c['scratch'] += 1
        elif op.startswith('s_waitcnt'):
            c['waitcnt'] += 1
        elif op.startswith('s_'):
            c['salu'] += 1
    return c


def main():
    s = open(sys.argv[1]).read()
    body = kernel_body(s, sys.argv[2] if len(sys.argv) > 2 else 'k_stft_ola')
    lines = body.split('\n')
    labels = {}
    for i, l in enumerate(lines):
        mm = re.match(r'^(\.LBB\d+_\d+):', l)
        if mm:
            labels[mm.group(1)] = i
    loops = []
    for i, l in enumerate(lines):
        mm = re.search(r's_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)', l)
        if mm and mm.group(1) in labels and labels[mm.group(1)] < i:
            loops.append((labels[mm.group(1)], i, mm.group(1)))
    code = [l.strip() for l in lines if l.strip() and not l.strip().startswith(('.', ';'))]
    print('whole kernel', len(code), dict(mix(code)))
    for a, b, t in sorted(loops, key=lambda x: x[0] - x[1])[:8]:
        seg = [l.strip() for l in lines[a:b + 1]
               if l.strip() and not l.strip().startswith(('.', ';'))]
        print(t, a, b, len(seg), dict(mix(seg)))


if __name__ == '__main__':
    main()
