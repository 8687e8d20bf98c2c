#!/usr/bin/env python3
"""LDS bank-conflict model of the register FFT's four exchanges (tm_fft.h) for
P = 64 (n_fft 2048) and P = 128 (n_fft 4096), under the gfx950 lane-group /
bank rules (MI355X_MICROARCH.md "LDS"): an 8-byte access as ds_read_b64
(2 x 32 lanes, dword mod 64) or as ds_read2*/ds_write*_b64 (4 x 16 lanes,
dword mod 32).  Prints the extra LDS cycles per frame and wave for each
exchange and form; tm_fft.h's x2col must give zero for the forms hipcc emits
(check the kernel's assembly: tools/isa_loopbody.py)."""


def g_of(P):
    if P > 64:
        return lambda c: ((c >> 1) & 7) ^ ((c & 1) << 2)
    return lambda c: c & 7


def conflicts(addrs, groups, nb):
    extra = 0
    for grp in groups:
        banks = {}
        for lane in grp:
            for d in addrs[lane]:
                banks.setdefault(d % nb, set()).add(d)
        extra += max(len(v) for v in banks.values()) - 1
    return extra


FORMS = {"b64 (2x32, mod 64)": ([list(range(0, 32)), list(range(32, 64))], 64),
         "b64 merged / write (4x16, mod 32)": ([list(range(i, i + 16)) for i in range(0, 64, 16)], 32)}


def exchange_conflicts(P):
    PB, RW, g = P // 8, P + 8, g_of(P)
    x2 = lambda a, c: 8 * c + (a ^ g(c))
    ex = {"x1 write (K*RW + L)": lambda L, K: K * RW + L,
          "x1 read / x4 write (q*RW + a + 8b)": lambda L, K: (L >> 3) * RW + (L & 7) + 8 * K,
          "x2 write / x3 read (q*RW + x2col(a, c))": lambda L, K: (L >> 3) * RW + x2(L & 7, K),
          "x2 read / x3 write (row*RW + x2col(A, c))":
              lambda L, K: ((L // PB) + 8 * (K // 8)) * RW + x2(K % 8, L % PB)}
    out = {}
    for name, f in ex.items():
        for form, (groups, nb) in FORMS.items():
            e = 0
            for w in range(P // 64):
                for K in range(PB):
                    ad = [[2 * f(64 * w + l, K), 2 * f(64 * w + l, K) + 1] for l in range(64)]
                    e += conflicts(ad, groups, nb)
            out[(name, form)] = e
    return out


if __name__ == "__main__":
    for P in (64, 128):
        for (name, form), e in exchange_conflicts(P).items():
            print(f"P={P:3d}  {name:44s} {form:34s} extra cycles/round {e}")
