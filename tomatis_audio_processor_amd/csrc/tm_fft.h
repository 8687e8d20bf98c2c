// tm_fft.h — N = 32*P point complex FFT held in registers of P lanes
// (32 complex values per lane), exchanged through LDS, for gfx950 wave64.
//
// Decomposition (four-step, then the P-point step split 8 x PB):
//   n = n1 + P*n2            (n1 = lane, n2 = register)         step 1: DFT_32 over n2
//   twiddle W_N^{n1*k2}                                          step 2
//   n1 = a + 8*b, k1 = c + PB*d, k = k2 + 32*k1
//   step 3a: DFT_PB over b   lanes (a = L%8, q = L/8), regs (j, b), k2 = q + PB*j
//   step 3b: twiddle W_P^{a*c}
//   step 3c: DFT_8 over a    lanes (c = L%PB, q' = L/PB), regs (j', d), k2 = q' + 8*j'
// After the forward transform lane (c, q') register j'*8+d holds bin
//   k = (q' + 8 j') + 32 (c + PB d).
// The inverse walks the same steps backwards with conjugate twiddles and ends
// with lane L register n2 holding sample L + P*n2 (the OLA-friendly layout).
// Exchanges go through an LDS round buffer of PB rows x (P+8) complex; rounds
// cover k2 blocks of PB so a round reads back exactly the registers it wrote.
#pragma once
#include "tm_common.h"
#include "../../include/tomatis_hip.h"  // TOMATIS_ERR_* bits

namespace tdsp {

template <int P_, int NR_ = 32>
struct FftGeo {
  static constexpr int P = P_;
  static constexpr int NR = NR_;            // complex registers per lane
  static constexpr int N = NR * P;          // transform size
  static constexpr int PB = P / 8;          // step-3a size
  static constexpr int NJ = NR / PB;        // step-3a transforms per lane
  static constexpr int RW = P + 8;          // LDS row stride (complex)
  static constexpr int ROUNDS = NR / PB;    // exchange rounds
  static constexpr int BUF = PB * RW;       // complex per round buffer
  // LDS per sequence: the round buffer, then (P > 64) one slot holding the
  // pair-barrier counter of the sequence's two waves
  static constexpr int SEQ_LDS = BUF + (P > 64 ? 1 : 0);
  static_assert(PB >= 4 && PB <= NR && NR % 8 == 0, "need 4 <= P/8 <= NR, NR % 8 == 0");
};

// Barrier of the two waves of a P = 128 sequence (not the whole workgroup):
// a counter in the sequence's LDS slot.  Both waves add 1 per barrier and can
// be at most one barrier apart, so the old value o of barrier k is 2k or
// 2k + 1 and the barrier completes when the counter reaches 2k + 2.  LDS
// operations of a wave execute in order, so the writes before the add are
// visible to the partner's reads after its poll.  Bounded spin: a stuck
// partner sets the error flag instead of hanging the GPU.
// Straight-line for the register allocator (a compiled spin loop and the
// lane-0 branch between the exchange rounds of a kernel at 256 VGPRs made it
// spill): lane 0's add (EXEC narrowed inside the asm) and the poll loop are one
// inline-asm block; returns false on a timeout, which the caller reports.
__device__ __forceinline__ bool pair_wait(uint32_t* ctr) {
  const uint32_t addr =
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)ctr;  // LDS offset
  uint32_t c, d, t;
  uint64_t ex;
  int left = 1 << 22;
  __asm__ volatile(
      "  s_waitcnt lgkmcnt(0)\n"            // this wave's exchange writes have landed
      "  s_mov_b64 %[ex], exec\n"
      "  s_mov_b64 exec, 1\n"
      "  ds_add_rtn_u32 %[c], %[a], %[one]\n"
      "  s_waitcnt lgkmcnt(0)\n"
      "  s_mov_b64 exec, %[ex]\n"
      "  v_readfirstlane_b32 %[t], %[c]\n"
      "  s_and_b32 %[t], %[t], -2\n"
      "  s_add_u32 %[t], %[t], 2\n"         // target = (old & ~1) + 2
      "1:\n"
      "  ds_read_b32 %[c], %[a]\n"
      "  s_waitcnt lgkmcnt(0)\n"
      "  v_readfirstlane_b32 %[d], %[c]\n"
      "  s_sub_u32 %[d], %[d], %[t]\n"
      "  s_cmp_gt_i32 %[d], -1\n"          // (int)(counter - target) >= 0: done
      "  s_cbranch_scc1 2f\n"
      "  s_sub_u32 %[n], %[n], 1\n"
      "  s_cmp_eq_u32 %[n], 0\n"
      "  s_cbranch_scc1 2f\n"
      "  s_sleep 1\n"
      "  s_branch 1b\n"
      "2:\n"
      : [c] "=&v"(c), [d] "=&s"(d), [t] "=&s"(t), [ex] "=&s"(ex), [n] "+s"(left)
      : [a] "v"(addr), [one] "v"(1u)
      : "scc", "memory");
  return left != 0;
}
__device__ __forceinline__ void pair_barrier(uint32_t* ctr, uint32_t* err) {
  if (!pair_wait(ctr) && err && (threadIdx.x & 63) == 0) atomicOr(err, TOMATIS_ERR_PAIR_BARRIER);
}

// LDS synchronisation for an exchange: wave-local when P == 64, the pair
// barrier when P == 128 (counter at buf[BUF]), else the workgroup barrier.
template <int P, int NR = 32>
__device__ __forceinline__ void xsync(cf* buf = nullptr, uint32_t* err = nullptr) {
  if constexpr (P == 128) {
    pair_barrier(reinterpret_cast<uint32_t*>(buf + FftGeo<P, NR>::BUF), err);
    return;
  }
  if constexpr (P <= 64) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  } else {
    __syncthreads();
  }
}

// exchange-2 column of element (a, c) in a row: XOR swizzle a ^ g(c).
// P = 64 (c < 8): g(c) = c.  P = 128 (c < 16): the exchange-2 reads and
// exchange-3 writes of one element index go out as ds_read2st64_b64 /
// ds_write2st64_b64 (the two rounds' rows in one instruction), whose 16-lane
// groups (c = 0..15 at one row) bank by dword mod 32, i.e. by
// (c & 1, a ^ g(c)): g must be a bijection on the even and on the odd c.
// g(c) = (c >> 1) ^ 4 (c & 1) is (plain c & 7 maps c and c + 8 onto the same
// banks: 2-way conflicts, 16.5 % of the LDS cycles of C5x).  The other
// exchange instructions bank on (q, a) and are conflict-free for any g
// (tools/lds_banks.py checks every exchange against the gfx950 lane-group /
// bank rules, MI355X_MICROARCH.md "LDS").
template <int P>
__device__ __forceinline__ int x2col(int a, int c) {
  if constexpr (P > 64) return 8 * c + (a ^ (((c >> 1) & 7) ^ ((c & 1) << 2)));
  return 8 * c + (a ^ (c & 7));
}

// forward FFT.  v: 32 registers (input x[L + P*n2]); out: bin layout above.
// twN: LDS W_N^{n1*k2} in lane-pair layout [k2/2][n1][k2&1] (16-B aligned);
// twP: LDS [P] with W_P^m; buf: round buffer.
// LT: twP is the per-lane table W_P^{(L%8)*m} for m < 8 in lane-pair layout
// [m/2][L][m&1] (P == 64 only: one ds_read_b128 per two twiddles, one address
// VGPR instead of seven)
template <int P, int NR = 32, bool LT = false>
__device__ __forceinline__ void fft_fwd(cf (&v)[NR], int L, const cf* twN, const cf* twP,
                                        cf* buf, uint32_t* err = nullptr) {
  using G = FftGeo<P, NR>;
  constexpr int PB = G::PB, RW = G::RW;
  const int a1 = L & 7, q1 = L >> 3;
  const int c3 = L % PB, q3 = L / PB;
  // step 1 (outputs carry splan<NR, 0>().sig: the twN table absorbs them)
  sdft<NR, 0, 0, NR>(v);
  // step 2 (twiddles in lane-pair layout: one ds_read_b128 per two registers)
  sfor<0, NR / 2>([&](auto kk) {
    constexpr int K2 = decltype(kk)::value;
    const float4 t = reinterpret_cast<const float4*>(twN)[K2 * P + L];
    if constexpr (K2 > 0) v[2 * K2] = cmul(v[2 * K2], cf{t.x, t.y});
    v[2 * K2 + 1] = cmul(v[2 * K2 + 1], cf{t.z, t.w});
  });
  // exchange 1 : (lane n1, reg k2) -> (lane (a,q), reg (j,b))
  sfor<0, G::ROUNDS>([&](auto rr) {
    constexpr int R = decltype(rr)::value;
    sfor<0, PB>([&](auto kk) {
      constexpr int K = decltype(kk)::value;
      buf[K * RW + L] = v[R * PB + K];
    });
    xsync<P, NR>(buf, err);
    sfor<0, PB>([&](auto bb) {
      constexpr int B = decltype(bb)::value;
      v[R * PB + B] = buf[q1 * RW + a1 + 8 * B];
    });
    xsync<P, NR>(buf, err);
  });
  // step 3a: DFT_PB over b for each j (output c carries splan<PB, 0>().sig[c],
  // absorbed by the step-3b twiddles)
  sfor<0, G::NJ>([&](auto jj) {
    constexpr int J = decltype(jj)::value;
    sdft<PB, 0, J * PB, NR>(v);
  });
  // step 3b: W_P^{a c}
  if constexpr (LT) {
    static_assert(PB == 8, "lane twiddle table needs P == 64");
    sfor<0, 4>([&](auto cc) {
      constexpr int C2 = decltype(cc)::value;
      const float4 t = reinterpret_cast<const float4*>(twP)[C2 * P + L];
      sfor<0, G::NJ>([&](auto jj) {
        constexpr int J = decltype(jj)::value;
        if constexpr (C2 > 0) v[J * PB + 2 * C2] = cmul(v[J * PB + 2 * C2], cf{t.x, t.y});
        v[J * PB + 2 * C2 + 1] = cmul(v[J * PB + 2 * C2 + 1], cf{t.z, t.w});
      });
    });
  } else {
    sfor<1, PB>([&](auto cc) {
      constexpr int C = decltype(cc)::value;
      constexpr float sc = (float)splan<PB, 0>().sig[C];
      const cf w = cscale(twP[(a1 * C) & (P - 1)], sc);
      sfor<0, G::NJ>([&](auto jj) {
        constexpr int J = decltype(jj)::value;
        v[J * PB + C] = cmul(v[J * PB + C], w);
      });
    });
  }
  // exchange 2 : (lane (a,q), reg (j,c)) -> (lane (c,q'), reg (j',a))
  sfor<0, G::ROUNDS>([&](auto rr) {
    constexpr int R = decltype(rr)::value;
    sfor<0, PB>([&](auto cc) {
      constexpr int C = decltype(cc)::value;
      buf[q1 * RW + x2col<P>(a1, C)] = v[R * PB + C];
    });
    xsync<P, NR>(buf, err);
    sfor<0, PB / 8>([&](auto jj) {
      constexpr int JJ = decltype(jj)::value;
      const int row = q3 + 8 * JJ;
      sfor<0, 8>([&](auto aa) {
        constexpr int A = decltype(aa)::value;
        v[R * PB + JJ * 8 + A] = buf[row * RW + x2col<P>(A, c3)];
      });
    });
    xsync<P, NR>(buf, err);
  });
  // step 3c: DFT_8 over a (output d carries splan<8, 0>().sig[d], absorbed by
  // the per-lane gain rows, k_gain_perm)
  sfor<0, NR / 8>([&](auto jj) {
    constexpr int J = decltype(jj)::value;
    sdft<8, 0, J * 8, NR>(v);
  });
}

// inverse (unnormalised) FFT: bin layout -> v[n2] = x[L + P*n2] * N
template <int P, int NR = 32, bool LT = false>
__device__ __forceinline__ void fft_inv(cf (&v)[NR], int L, const cf* twN, const cf* twP,
                                        cf* buf, uint32_t* err = nullptr) {
  using G = FftGeo<P, NR>;
  constexpr int PB = G::PB, RW = G::RW;
  const int a1 = L & 7, q1 = L >> 3;
  const int c3 = L % PB, q3 = L / PB;
  // step 3c': IDFT_8 over d -> a (output a carries splan<8, 1>().sig[a] =
  // splan<8, 0>().sig[a]: absorbed by the scaled step-3b' twiddles; P = 64: the
  // forward's own table, PB = 8)
  sfor<0, NR / 8>([&](auto jj) {
    constexpr int J = decltype(jj)::value;
    sdft<8, 1, J * 8, NR>(v);
  });
  // step 3b': conj W_P^{a c3}
  if constexpr (LT) {  // c3 = L % 8 here: same table as the forward step 3b
    sfor<0, 4>([&](auto aa) {
      constexpr int A2 = decltype(aa)::value;
      const float4 t = reinterpret_cast<const float4*>(twP)[A2 * P + L];
      sfor<0, NR / 8>([&](auto jj) {
        constexpr int J = decltype(jj)::value;
        if constexpr (A2 > 0) v[J * 8 + 2 * A2] = cmulc(v[J * 8 + 2 * A2], cf{t.x, t.y});
        v[J * 8 + 2 * A2 + 1] = cmulc(v[J * 8 + 2 * A2 + 1], cf{t.z, t.w});
      });
    });
  } else {
    sfor<1, 8>([&](auto aa) {
      constexpr int A = decltype(aa)::value;
      constexpr float sc = (float)splan<8, 1>().sig[A];
      const cf w = cscale(twP[(A * c3) & (P - 1)], sc);
      sfor<0, NR / 8>([&](auto jj) {
        constexpr int J = decltype(jj)::value;
        v[J * 8 + A] = cmulc(v[J * 8 + A], w);
      });
    });
  }
  // exchange 3 : (lane (c,q'), reg (j',a)) -> (lane (a,q), reg (j,c))
  sfor<0, G::ROUNDS>([&](auto rr) {
    constexpr int R = decltype(rr)::value;
    sfor<0, PB / 8>([&](auto jj) {
      constexpr int JJ = decltype(jj)::value;
      const int row = q3 + 8 * JJ;
      sfor<0, 8>([&](auto aa) {
        constexpr int A = decltype(aa)::value;
        buf[row * RW + x2col<P>(A, c3)] = v[R * PB + JJ * 8 + A];
      });
    });
    xsync<P, NR>(buf, err);
    sfor<0, PB>([&](auto cc) {
      constexpr int C = decltype(cc)::value;
      v[R * PB + C] = buf[q1 * RW + x2col<P>(a1, C)];
    });
    xsync<P, NR>(buf, err);
  });
  // step 3a': IDFT_PB over c -> b
  sfor<0, G::NJ>([&](auto jj) {
    constexpr int J = decltype(jj)::value;
    dft<PB, true, J * PB, 1, NR>(v);
  });
  // exchange 4 : (lane (a,q), reg (j,b)) -> (lane n1, reg k2)
  sfor<0, G::ROUNDS>([&](auto rr) {
    constexpr int R = decltype(rr)::value;
    sfor<0, PB>([&](auto bb) {
      constexpr int B = decltype(bb)::value;
      buf[q1 * RW + a1 + 8 * B] = v[R * PB + B];
    });
    xsync<P, NR>(buf, err);
    sfor<0, PB>([&](auto kk) {
      constexpr int K = decltype(kk)::value;
      v[R * PB + K] = buf[K * RW + L];
    });
    xsync<P, NR>(buf, err);
  });
  // step 2': conj W_N^{n1 k2}
  sfor<0, NR / 2>([&](auto kk) {
    constexpr int K2 = decltype(kk)::value;
    const float4 t = reinterpret_cast<const float4*>(twN)[K2 * P + L];
    if constexpr (K2 > 0) v[2 * K2] = cmulc(v[2 * K2], cf{t.x, t.y});
    v[2 * K2 + 1] = cmulc(v[2 * K2 + 1], cf{t.z, t.w});
  });
  // step 1': IDFT_NR over k2 -> n2.  The scaled twN table multiplied register
  // k2 by splan<NR, 0>().sig[k2] on top of the twiddle, so the inputs carry
  // 1 / that (plan 2); the outputs carry splan<NR, 2>().sig[n2], absorbed by
  // the synthesis window (winS).
  sdft<NR, 2, 0, NR>(v);
}

// ---------------------------------------------------------------------------
// Single-exchange FFT (P = 64, NR = 32: n_fft 2048).  Same four-step split
// n = n1 + 64 n2, k = k2 + 32 k1 as above; the 64-point DFT over the lane
// index n1 = m + 32 b is done as one radix-2 stage over lane bit 5 followed by
// a 32-point register DFT, so a direction needs ONE LDS exchange instead of two:
//   step 3a (lane bit 5 -> register bit): v_permlane32_swap of register pairs
//     (2j, 2j+1): lane (m, s) then holds Y[m + 32 b, k2 = 2j + s] in register
//     2j + b; the DIF butterfly over b gives U_e = W_64^{m e} (Y[m] + (-1)^e Y[m+32])
//     in register 2j + e (one per-lane twiddle W_64^m, on the e = 1 registers);
//   exchange (one float component at a time, 8.5 KB per wave): every register r
//     is written as one LDS row by ds_write_addtid_b32 (lane-contiguous, no
//     address VGPR: the fastest LDS store form, MI355X_MICROARCH.md "LDS"), and
//     lane (r', s') reads row r' columns 32 s' .. 32 s' + 31 with eight
//     conflict-free ds_read_b128 (row pitch 68 floats);
//   step 3b: DFT_32 over m in registers.
// After the forward transform lane L (r = L & 31, s = L >> 5) register i holds
// bin k = (2 (r >> 1) + s) + 32 (r & 1) + 64 i with scale splan<32, 0>().sig[i].
// The inverse walks back; its first DFT's output scales splan<32, 1>().sig[m]
// stay on lane m (= L & 31) through the exchange and the butterflies and are
// absorbed by the synthesis window (host table winS).
// ---------------------------------------------------------------------------
constexpr int kXPitch = 68;           // floats per exchange row (bank rotation 4)
constexpr int kXBuf = 32 * kXPitch;   // floats per sequence

__device__ __forceinline__ void swap32(cf& a, cf& b) {  // lanes 32..63 of a <-> lanes 0..31 of b
  const auto rx = __builtin_amdgcn_permlane32_swap(__float_as_uint(a.x), __float_as_uint(b.x), false, false);
  const auto ry = __builtin_amdgcn_permlane32_swap(__float_as_uint(a.y), __float_as_uint(b.y), false, false);
  a = {__uint_as_float(rx[0]), __uint_as_float(ry[0])};
  b = {__uint_as_float(rx[1]), __uint_as_float(ry[1])};
}

// eight rows of one component: ds_write_addtid_b32 at M0 + offset + 4 lane.
// M0 is set inside the block (a SALU write of M0 needs one wait state before
// an add-TID LDS instruction) and listed as clobbered, so a value the compiler
// keeps in M0 (LDS-DMA set-up) is re-materialised after it (clang warns that a
// reserved register is not saved around the statement: nothing needs saving).
#define TM_ADDTID8(C, R0)                                                           \
  _Pragma("clang diagnostic push") _Pragma("clang diagnostic ignored \"-Winline-asm\"") \
  __asm__ volatile(                                                                 \
      "s_mov_b32 m0, %8\n\ts_nop 0\n\t"                                             \
      "ds_write_addtid_b32 %0 offset:%9\n\tds_write_addtid_b32 %1 offset:%10\n\t"    \
      "ds_write_addtid_b32 %2 offset:%11\n\tds_write_addtid_b32 %3 offset:%12\n\t"   \
      "ds_write_addtid_b32 %4 offset:%13\n\tds_write_addtid_b32 %5 offset:%14\n\t"   \
      "ds_write_addtid_b32 %6 offset:%15\n\tds_write_addtid_b32 %7 offset:%16"       \
      ::"v"(v[R0].C), "v"(v[R0 + 1].C), "v"(v[R0 + 2].C), "v"(v[R0 + 3].C),          \
      "v"(v[R0 + 4].C), "v"(v[R0 + 5].C), "v"(v[R0 + 6].C), "v"(v[R0 + 7].C),        \
      "s"(base), "n"((R0) * kXPitch * 4), "n"((R0 + 1) * kXPitch * 4),                \
      "n"((R0 + 2) * kXPitch * 4), "n"((R0 + 3) * kXPitch * 4),                       \
      "n"((R0 + 4) * kXPitch * 4), "n"((R0 + 5) * kXPitch * 4),                       \
      "n"((R0 + 6) * kXPitch * 4), "n"((R0 + 7) * kXPitch * 4)                        \
      : "memory", "m0") _Pragma("clang diagnostic pop")

// transpose (lane, register) through LDS: register r of lane (m, s) -> register
// m of lane (r, s).  buf: this wave's kXBuf floats (16-B aligned).  LDS
// operations of one wave complete in order, so each read sees the rows written
// before it and the second component's writes land after the first's reads;
// the "memory" clobbers keep the compiler's LDS reads after the writes.
__device__ __forceinline__ void xchg32(cf (&v)[32], float* buf, int L) {
  const uint32_t base = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float*)buf);
  const float4* rp = reinterpret_cast<const float4*>(buf + (L & 31) * kXPitch + 32 * (L >> 5));
  TM_ADDTID8(x, 0);
  TM_ADDTID8(x, 8);
  TM_ADDTID8(x, 16);
  TM_ADDTID8(x, 24);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float4 t = rp[q];
    v[4 * q].x = t.x;
    v[4 * q + 1].x = t.y;
    v[4 * q + 2].x = t.z;
    v[4 * q + 3].x = t.w;
  }
  TM_ADDTID8(y, 0);
  TM_ADDTID8(y, 8);
  TM_ADDTID8(y, 16);
  TM_ADDTID8(y, 24);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float4 t = rp[q];
    v[4 * q].y = t.x;
    v[4 * q + 1].y = t.y;
    v[4 * q + 2].y = t.z;
    v[4 * q + 3].y = t.w;
  }
}
#undef TM_ADDTID8

// step 1 + step 2 of the forward (P lanes: twN is [NR/2][P] lane pairs)
// (P = 128: register 0 of wave 1 holds k2 = 16, whose twiddle is not 1)
template <int P>
__device__ __forceinline__ void fftx_head(cf (&v)[32], int L, const cf* twN) {
  constexpr int NR = 32;
  sdft<NR, 0, 0, NR>(v);
  sfor<0, NR / 2>([&](auto kk) {
    constexpr int K2 = decltype(kk)::value;
    const float4 t = reinterpret_cast<const float4*>(twN)[K2 * P + L];
    if constexpr (K2 > 0 || P > 64) v[2 * K2] = cmul(v[2 * K2], cf{t.x, t.y});
    v[2 * K2 + 1] = cmul(v[2 * K2 + 1], cf{t.z, t.w});
  });
}
// the 64-point DFT over the wave's lanes of each of the 32 registers (lane
// bit 5 by permlane32 + butterfly, then the transpose and DFT_32): register r
// of lane l -> lane (r', s) (r' = l & 31, s = l >> 5) register i holds
// output k1 = (r' & 1) + 2 i of the DFT of register r = 2 (r' >> 1) + s.
// l5: this lane's index within the wave (L & 63); w: W_64^{l5 & 31}
__device__ __forceinline__ void fftx_tail(cf (&v)[32], int l5, cf w, float* buf) {
  constexpr int NR = 32;
  sfor<0, NR / 2>([&](auto jj) {
    constexpr int J = decltype(jj)::value;
    swap32(v[2 * J], v[2 * J + 1]);
    const cf a = v[2 * J], b = v[2 * J + 1];
    v[2 * J] = a + b;
    v[2 * J + 1] = cmul(a - b, w);
  });
  xchg32(v, buf, l5);
  sdft<NR, 0, 0, NR>(v);
}
// inverse of fftx_tail (unnormalised); the outputs carry splan<32, 1>().sig[l5 & 31]
__device__ __forceinline__ void fftx_itail(cf (&v)[32], int l5, cf w, float* buf) {
  constexpr int NR = 32;
  sdft<NR, 1, 0, NR>(v);
  xchg32(v, buf, l5);
  sfor<0, NR / 2>([&](auto jj) {
    constexpr int J = decltype(jj)::value;
    const cf z0 = v[2 * J], z1 = cmulc(v[2 * J + 1], w);
    v[2 * J] = z0 + z1;
    v[2 * J + 1] = z0 - z1;
    swap32(v[2 * J], v[2 * J + 1]);
  });
}
// inverse of fftx_head: conj step 2, then DFT_32 (plan 2) over k2 -> n2
template <int P>
__device__ __forceinline__ void fftx_ihead(cf (&v)[32], int L, const cf* twN) {
  constexpr int NR = 32;
  sfor<0, NR / 2>([&](auto kk) {
    constexpr int K2 = decltype(kk)::value;
    const float4 t = reinterpret_cast<const float4*>(twN)[K2 * P + L];
    if constexpr (K2 > 0 || P > 64) v[2 * K2] = cmulc(v[2 * K2], cf{t.x, t.y});
    v[2 * K2 + 1] = cmulc(v[2 * K2 + 1], cf{t.z, t.w});
  });
  sdft<NR, 2, 0, NR>(v);
}

// forward: v[n2] = x[L + 64 n2] -> bin layout above.  twN: the step-2 table
// (lane-pair layout, as fft_fwd); w: W_64^{L & 31}.
__device__ __forceinline__ void fftx_fwd(cf (&v)[32], int L, const cf* twN, cf w, float* buf) {
  fftx_head<64>(v, L, twN);
  fftx_tail(v, L, w, buf);
}

// inverse (unnormalised): bin layout -> v[n2] = N x[L + 64 n2] / (sig1[L & 31] sig2[n2])
__device__ __forceinline__ void fftx_inv(cf (&v)[32], int L, const cf* twN, cf w, float* buf) {
  fftx_itail(v, L, w, buf);
  fftx_ihead<64>(v, L, twN);
}

// bin index held by lane L, register i after fftx_fwd
__device__ __forceinline__ int fftx_bin(int L, int i) {
  const int r = L & 31, s = L >> 5;
  return (2 * (r >> 1) + s) + 32 * (r & 1) + 64 * i;
}

// ---------------------------------------------------------------------------
// n_fft 4096 on two waves (P = 128 lanes L = l + 64 w, 32 registers: sample
// L + 128 n2).  Steps 1-2 as above per lane; the 128-point DFT over L = m + 64 w
// starts with the radix-2 stage over the wave bit: wave w keeps k2 in
// [16 w, 16 w + 16) and trades the other half with its partner through LDS
// (8 KB each way, one pair barrier).  Wave 1 works with its k2 rotated by 16
// (register r holds k2 = (r + 16) mod 32): its analysis window carries
// (-1)^n2 (DFT_32 of x (-1)^n2 is X[k2 + 16]), its step-2 table row r the
// twiddle of that k2, its synthesis window (-1)^n2 again -- so both waves send
// registers 16..31 and receive into them, with no wave-dependent register
// index.  After the trade register j holds Y[m, k2] and 16 + j holds
// Y[m + 64, k2] in wave 0, the reverse in wave 1 (k2 = 16 w + j), so the
// butterfly U_0 = v[j] + v[16 + j], U_1 = (v[j] - v[16 + j]) W_128^m takes
// -W_128^m in wave 1 (twiddle table s_twP: W_128^{l} (1 - 2 w)).  Then each
// wave runs fftx_tail's 64-point DFT over m on its 32 registers (j, 16 + j:
// e = 0, 1).  Bin of lane L (w, l: r' = l & 31, s = l >> 5), register i:
// r = 2 (r' >> 1) + s, k = (16 w + (r & 15)) + 32 (r >> 4) + 64 ((r' & 1) + 2 i).
// LDS: two kXBuf-float regions H_0, H_1 (+ the pair-barrier counter).  Wave w
// sends through its own region H_w and then runs its exchanges in H_{1-w};
// on the way back it sends through H_{1-w}: no region is written while the
// partner may still read it, with two pair barriers per frame.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void x128_trade(cf (&v)[32], int l, float* out, const float* in,
                                           uint32_t* ctr, uint32_t* err) {
  float2* o = reinterpret_cast<float2*>(out) + l;
  const float2* q = reinterpret_cast<const float2*>(in) + l;
  // the partner wave waits at this pair barrier: the trade runs at raised
  // priority (c5x kernel -1.4 %, DESIGN.md §6 "Wave priority")
  __builtin_amdgcn_s_setprio(2);
  sfor<0, 16>([&](auto jj) {
    constexpr int J = decltype(jj)::value;
    o[64 * J] = make_float2(v[16 + J].x, v[16 + J].y);
  });
  pair_barrier(ctr, err);
  sfor<0, 16>([&](auto jj) {
    constexpr int J = decltype(jj)::value;
    const float2 t = q[64 * J];
    v[16 + J] = {t.x, t.y};
  });
  __builtin_amdgcn_s_setprio(0);
}

// forward.  buf: the sequence's 2 kXBuf regions (H_0, H_1) then the counter;
// w128: W_128^{l} (1 - 2 w) (l = L & 63); w64: W_64^{l & 31}
__device__ __forceinline__ void fftx128_fwd(cf (&v)[32], int L, const cf* twN, cf w128, cf w64,
                                            float* buf, uint32_t* err) {
  const int l = L & 63, w = __builtin_amdgcn_readfirstlane(L >> 6);
  uint32_t* ctr = reinterpret_cast<uint32_t*>(buf + 2 * kXBuf);
  float* const hw = buf + w * kXBuf;
  float* const ho = buf + (1 - w) * kXBuf;
  fftx_head<128>(v, L, twN);
  x128_trade(v, l, hw, ho, ctr, err);
  sfor<0, 16>([&](auto jj) {
    constexpr int J = decltype(jj)::value;
    const cf a = v[J], b = v[16 + J];
    v[J] = a + b;
    v[16 + J] = cmul(a - b, w128);
  });
  fftx_tail(v, l, w64, ho);
}

// inverse: bin layout -> v[n2] = N x[L + 128 n2] (-1)^{w n2} / (sig1[l & 31] sig2[n2])
__device__ __forceinline__ void fftx128_inv(cf (&v)[32], int L, const cf* twN, cf w128, cf w64,
                                            float* buf, uint32_t* err) {
  const int l = L & 63, w = __builtin_amdgcn_readfirstlane(L >> 6);
  uint32_t* ctr = reinterpret_cast<uint32_t*>(buf + 2 * kXBuf);
  float* const hw = buf + w * kXBuf;
  float* const ho = buf + (1 - w) * kXBuf;
  fftx_itail(v, l, w64, ho);
  // wave 0: v[j] = b 0 (kept), v[16 + j] = b 1 (wave 1's register 16 + j);
  // wave 1 (twiddle negated): v[j] = b 1 (kept), v[16 + j] = b 0 (wave 0's)
  sfor<0, 16>([&](auto jj) {
    constexpr int J = decltype(jj)::value;
    const cf z0 = v[J], z1 = cmulc(v[16 + J], w128);
    v[J] = z0 + z1;
    v[16 + J] = z0 - z1;
  });
  x128_trade(v, l, ho, hw, ctr, err);
  fftx_ihead<128>(v, L, twN);
}

__device__ __forceinline__ int fftx128_bin(int L, int i) {
  const int w = L >> 6, l = L & 63, rp = l & 31, s = l >> 5;
  const int r = 2 * (rp >> 1) + s;
  return (16 * w + (r & 15)) + 32 * (r >> 4) + 64 * ((rp & 1) + 2 * i);
}

// per-lane register tables (window, gains, 1/wsum) in lane-quad layout:
// element (register i, lane L) at ((i/4)*P + L)*4 + i%4, read with ds_read_b128
template <int P>
__device__ __forceinline__ constexpr int lq(int i, int L) {
  return ((i >> 2) * P + L) * 4 + (i & 3);
}

// bin index held by lane L, register index i (= j'*8 + d) after fft_fwd
template <int P, int NR = 32>
__device__ __forceinline__ int fft_bin(int L, int i) {
  constexpr int PB = P / 8;
  const int c3 = L % PB, q3 = L / PB;
  const int jp = i >> 3, d = i & 7;
  return (q3 + 8 * jp) + NR * (c3 + PB * d);
}

}  // namespace tdsp
