// Fragment / region helpers of the key-major dK/dV passes with 64 keys per wave and AGPR dK / dV
// accumulators, shared by attention_dkdv6.hip (dkdv6/7/8) and attention_bwd1.hip (the one-pass
// backward).  Device-only inline code; the including file is compiled with
// -mllvm -amdgpu-mfma-vgpr-form (Makefile).
#pragma once
#include <type_traits>

#include "attn_frag.h"

namespace {

// acc += x . b  (32x32x16, accumulator in AGPRs).  NOP: open with s_nop 1, for a B operand that a
// VALU instruction may have written right before (the compiler pads no hazard into an asm statement)
template <typename T, bool NOP>
__device__ __forceinline__ void mfma_acc(f32x16& acc, const typename Mfma<T>::frag& x, const typename Mfma<T>::frag& b) {
    if constexpr (std::is_same<T, bf16>::value) {
        if constexpr (NOP)
            asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(x), "v"(b));
        else
            asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(x), "v"(b));
    } else {
        if constexpr (NOP)
            asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(x), "v"(b));
        else
            asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(x), "v"(b));
    }
}

// nothing is scheduled across it: the regions below are issued in source order
__device__ __forceinline__ void fence() { __builtin_amdgcn_sched_barrier(0); }

template <typename T>
struct K6 {
    typedef typename Mfma<T>::frag frag;
    frag kf[2][4], vf[2][4];   // this wave's two 32-key blocks (B operands of the S / dP chains)
    f32x16 dk[2][2], dv[2][2];  // [block][d block]: dK^T / dV^T accumulators (AGPR)
};

// packed P / dS of one block as 16-bit B operands: word j of fragment s holds elements 8s+2j, +1
struct Packs {
    unsigned p[2][4], d[2][4];
};

template <typename T>
__device__ __forceinline__ typename Mfma<T>::frag as_frag(const unsigned (&w)[4]) {
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = {w[0], w[1], w[2], w[3]};
    return __builtin_bit_cast(typename Mfma<T>::frag, v);
}

// Q / dO row fragments (A operands of S and dP) of sub-slice `sub` of the slot at `base`
template <typename T>
__device__ __forceinline__ void load_qg(typename Mfma<T>::frag (&qa)[4], typename Mfma<T>::frag (&ga)[4],
                                        const char* base, int sub, int l32, int h) {
    const char* Qt = base + sub * 32 * 128;
    const char* Gt = base + 8192 + sub * 32 * 128;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        qa[s] = row_frag<T>(Qt, l32, 2 * s + h);
        ga[s] = row_frag<T>(Gt, l32, 2 * s + h);
    }
}

// transposed dO^T / Q^T fragments (A operands of dV^T += dO^T P, dK^T += Q^T dS)
template <typename T>
__device__ __forceinline__ void load_t(typename Mfma<T>::frag (&gt)[2][2], typename Mfma<T>::frag (&qt)[2][2],
                                       const char* base, int sub, int lane) {
    const char* Qt = base + sub * 32 * 128;
    const char* Gt = base + 8192 + sub * 32 * 128;
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int db = 0; db < 2; ++db) {
            gt[s][db] = tr_frag<T>(Gt, 0, s, db, lane);
            qt[s][db] = tr_frag<T>(Qt, 0, s, db, lane);
        }
}

// the S / dP accumulators of one block seeded with the sub-slice's -L and -DsScale delta (read
// straight from the slot's negated statistics)
__device__ __forceinline__ void seeds(f32x16& S, f32x16& P, const char* base, int sub, int h) {
    const float* Ls = (const float*)(base + 16384) + sub * 32;
    const float* Ds = Ls + 64;
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
        const f32x4 Lv = *(const f32x4*)(Ls + 8 * g4 + 4 * h);
        const f32x4 Dv = *(const f32x4*)(Ds + 8 * g4 + 4 * h);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            S[4 * g4 + e] = Lv[e];
            P[4 * g4 + e] = Dv[e];
        }
    }
}

// softmax VALU of elements 2i, 2i+1 of a block: P = exp2(S), dS = P dP', both packed
template <typename T>
__device__ __forceinline__ void fin_chunk(f32x16& S, f32x16& P, Packs& pk, int i) {
    typedef T t2 __attribute__((ext_vector_type(2)));
#ifdef DCLIP_DIAG_NOEXP  // timing probe: a 4-cycle multiply in place of the 8-cycle exp
    const float e0 = S[2 * i] * 0.5f;
    const float e1 = S[2 * i + 1] * 0.5f;
#else
    const float e0 = __builtin_amdgcn_exp2f(S[2 * i]);
    const float e1 = __builtin_amdgcn_exp2f(S[2 * i + 1]);
#endif
    const float d0 = e0 * P[2 * i], d1 = e1 * P[2 * i + 1];
    const t2 pp = {(T)e0, (T)e1};
    const t2 dd = {(T)d0, (T)d1};
    pk.p[i >> 2][i & 3] = __builtin_bit_cast(unsigned, pp);
    pk.d[i >> 2][i & 3] = __builtin_bit_cast(unsigned, dd);
}

}  // namespace
