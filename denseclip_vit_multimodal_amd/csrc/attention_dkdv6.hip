// Key-major dK/dV pass of the CLS-split attention backward with 64 keys per wave (one wave per
// SIMD), the dK / dV sums held in the accumulator (AGPR) file.
//
// Replaces the dK, dV half of the backward of nn.MultiheadAttention's softmax(q k^T d^-0.5) v
// (reference seg/denseclip/models.py:275, 287-289), the same arithmetic as
// attention.hip::attn_bwd_dkdv5_kernel: per key, dV = sum_q P[q][k] dO[q], dK = sum_q dS[q][k] q'
// with P = exp2(S - L) recomputed from the log2-domain lse and dS = P (dP - delta).
//
// Why a second kernel.  dkdv5 runs 32 keys per wave at two waves per SIMD: every Q / dO fragment
// it reads from LDS (and every -L / -delta seed) feeds ONE key block, so it issues 2.0 LDS
// instructions per MFMA and sits at 254 VGPRs with its fragment reads placed just before their
// MFMAs.  Here each wave owns 64 keys (two 32-key blocks): the Q / dO row fragments and the
// transposed Q^T / dO^T fragments of a 32-query sub-slice feed both blocks, which halves the LDS
// reads and the L2 -> LDS slice traffic per MFMA (a workgroup of 4 waves covers 256 keys).  The
// four dK / dV accumulators per block (128 registers) live in AGPRs: the dK / dV MFMAs are
// issued by inline asm with "+a" accumulator operands, and this file is compiled with
// -mllvm -amdgpu-mfma-vgpr-form so the compiler's own S / dP MFMAs keep their accumulators in
// arch VGPRs beside the softmax VALU (no v_accvgpr copies: the failure of the register-blocked
// variants measured in round 2).
//
// Issue order.  At one wave per SIMD nothing hides a stall, and hipcc's scheduler, which sees the
// asm statements as opaque, issued the regions back to back (all S / dP MFMAs, then all the softmax
// VALU, then the asm MFMAs).  The sub-slice is therefore written as four regions fenced by
// sched_barrier (sub6): the softmax VALU of one block sits between the MFMAs of the other, about
// six VALU instructions per 32-cycle MFMA gap.
//
// Hazards the compiler does not pad around an asm statement (cdna_hip_programming.md §5.7): a
// packed P / dS B-operand written by VALU just before an asm MFMA reads it -> that statement opens
// with s_nop 1 (only R4's first: everything else was packed a region earlier); the AGPR
// accumulators are read once, in the epilogue, behind an s_nop ladder inside a statement that
// names them.
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

// one 32-query sub-slice, four regions fenced in issue order (32 MFMAs):
//   R1  S / dP chains of block 0              (8)   | loads: gt / qt, block-1 seeds
//   R2  S / dP chains of block 1              (8)   | VALU: block 0's exp / mul / pack
//   R3  dV / dK of block 0 (asm, AGPR)        (8)   | VALU: block 1's exp / mul / pack; loads: next Q / dO
//   R4  dV / dK of block 1 (asm, AGPR)        (8)   | loads: next block-0 seeds
// S0 / P0 arrive seeded and qa / ga hold this sub-slice; both leave holding the next one (`nb`,
// `nsub`: the next sub-slice's slot and index)
template <typename T>
__device__ __forceinline__ void sub6(K6<T>& k, int h, int l32, int lane, const char* base, int sub, const char* nb,
                                     int nsub, typename Mfma<T>::frag (&qa)[4], typename Mfma<T>::frag (&ga)[4],
                                     f32x16& S0, f32x16& P0) {
    typedef typename Mfma<T>::frag frag;
    f32x16 S1, P1;
    frag gt[2][2], qt[2][2];
    Packs k0, k1;
    // ---- R1
    fence();
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        S0 = Mfma<T>::mma(qa[s], k.kf[0][s], S0);
        P0 = Mfma<T>::mma(ga[s], k.vf[0][s], P0);
    }
    load_t<T>(gt, qt, base, sub, lane);
    seeds(S1, P1, base, sub, h);
    fence();
    // ---- R2
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        S1 = Mfma<T>::mma(qa[s], k.kf[1][s], S1);
        fin_chunk<T>(S0, P0, k0, 2 * s);
        fence();
        P1 = Mfma<T>::mma(ga[s], k.vf[1][s], P1);
        fin_chunk<T>(S0, P0, k0, 2 * s + 1);
        fence();
    }
    // ---- R3
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        mfma_acc<T, false>(k.dv[0][0], gt[s][0], as_frag<T>(k0.p[s]));
        fin_chunk<T>(S1, P1, k1, 4 * s);
        fence();
        mfma_acc<T, false>(k.dv[0][1], gt[s][1], as_frag<T>(k0.p[s]));
        fin_chunk<T>(S1, P1, k1, 4 * s + 1);
        fence();
        mfma_acc<T, false>(k.dk[0][0], qt[s][0], as_frag<T>(k0.d[s]));
        fin_chunk<T>(S1, P1, k1, 4 * s + 2);
        fence();
        mfma_acc<T, false>(k.dk[0][1], qt[s][1], as_frag<T>(k0.d[s]));
        fin_chunk<T>(S1, P1, k1, 4 * s + 3);
        fence();
    }
    load_qg<T>(qa, ga, nb, nsub, l32, h);
    fence();
    // ---- R4
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        mfma_acc<T, true>(k.dv[1][0], gt[s][0], as_frag<T>(k1.p[s]));
        mfma_acc<T, false>(k.dv[1][1], gt[s][1], as_frag<T>(k1.p[s]));
        mfma_acc<T, false>(k.dk[1][0], qt[s][0], as_frag<T>(k1.d[s]));
        mfma_acc<T, false>(k.dk[1][1], qt[s][1], as_frag<T>(k1.d[s]));
    }
    seeds(S0, P0, nb, nsub, h);
    fence();
}

// one 64-query slice (two sub-slices), read one slice ahead as in attn_bwd_dkdv5_kernel: S0 / P0
// and qa / ga arrive holding (this slice, sub 0) and leave holding (next slice, sub 0)
template <typename T, int Q>
__device__ __forceinline__ void step6(Dkv2Ctx<T, 4>& c, K6<T>& k, int t, typename Mfma<T>::frag (&qa)[4],
                                      typename Mfma<T>::frag (&ga)[4], f32x16& S0, f32x16& P0) {
    typedef Dkv2Ctx<T, 4> X;
    // DCLIP_DIAG_* (tools/ab_attn.py timing probes only, never in the product build: the results
    // are wrong): NOWAIT skips the DMA wait, NOBAR the workgroup barrier
#ifndef DCLIP_DIAG_NOWAIT
    wait_vmcnt<X::PIECES + 1>();    // own pieces of slice t+1 landed (slice t+2 in flight)
#endif
#ifndef DCLIP_DIAG_NOBAR
    __builtin_amdgcn_s_barrier();  // everyone's; everyone done with step t-1 (slot (t+3) % 4 free)
#endif
    dkv2_issue<T, 4>(c, t + 3 < c.nt ? t + 3 : c.nt - 1, (Q + 3) & 3);
    const char* cur = c.smem + Q * X::SLOT;
    const char* nxt = c.smem + ((Q + 1) & 3) * X::SLOT;
    sub6<T>(k, c.h, c.l32, c.lane, cur, 0, cur, 1, qa, ga, S0, P0);
    sub6<T>(k, c.h, c.l32, c.lane, cur, 1, nxt, 0, qa, ga, S0, P0);
}

template <typename T>
__global__ __launch_bounds__(256, 1) void attn_bwd_dkdv6_kernel(const T* __restrict__ qkv, const T* __restrict__ dout,
                                                                const float* __restrict__ lse,
                                                                const float* __restrict__ delta,
                                                                const float* __restrict__ nlse,
                                                                const float* __restrict__ ndelta,
                                                                T* __restrict__ dqkv, int N, int H, float dk_scale,
                                                                float* __restrict__ r0q) {
    constexpr int NW = 4, KB = 64 * NW;
    typedef Dkv2Ctx<T, NW> X;
    typedef typename Mfma<T>::frag frag;
    // the ring, then the CLS-row fold's per-key weights dS_0 (used when r0q != null)
    __shared__ __attribute__((aligned(16))) char smem[4 * X::SLOT + KB * 4];
    X c;  // the LDS-DMA ring of Q / dO / statistics slices (its key-fragment members stay unused)
    K6<T> k;
    c.smem = smem;
    c.lane = threadIdx.x & 63;
    c.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    c.h = c.lane >> 5;
    c.l32 = c.lane & 31;
    const int nkb = (N - 1 + KB - 1) / KB;  // the last key block partial when N - 1 is ragged
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int kblk = tile % nkb, bh = tile / nkb, b = bh / H, hd = bh % H;
    const int C = H * HD;
    const int64_t ld = 3 * (int64_t)C;
    const T* Bb = qkv + (int64_t)b * N * ld;
    const T* dOb = dout + (int64_t)b * N * C;
    c.ldq = (uint32_t)(ld * sizeof(T));
    c.ldg = (uint32_t)(C * sizeof(T));
    c.nt = (N - 1 + 63) / 64;
    c.rem = N - 1 - 64 * (c.nt - 1);
    int key[2];
    bool kok[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
        key[kb] = 1 + kblk * KB + c.wave * 64 + kb * 32 + c.l32;
        kok[kb] = key[kb] < N;  // keys past N compute on key N - 1 and store nothing
        const int kc = kok[kb] ? key[kb] : N - 1;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            k.kf[kb][s] = *(const frag*)(Bb + (int64_t)kc * ld + C + hd * HD + (2 * s + c.h) * 8);
            k.vf[kb][s] = *(const frag*)(Bb + (int64_t)kc * ld + 2 * C + hd * HD + (2 * s + c.h) * 8);
        }
    }
    frag q0[4], g0[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        q0[s] = *(const frag*)(Bb + hd * HD + (2 * s + c.h) * 8);
        g0[s] = *(const frag*)(dOb + hd * HD + (2 * s + c.h) * 8);
    }
    typedef T t4 __attribute__((ext_vector_type(4)));
    t4 q0d[2][4], g0d[2][4];  // query 0's q and dO at this lane's accumulator rows d
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            q0d[db][g] = *(const t4*)(Bb + hd * HD + db * 32 + 8 * g + 4 * c.h);
            g0d[db][g] = *(const t4*)(dOb + hd * HD + db * 32 + 8 * g + 4 * c.h);
        }
    const float L0 = lse[(int64_t)bh * N], d0 = delta[(int64_t)bh * N];

    c.rs = make_rsrc(Bb, (uint32_t)N * c.ldq);
    c.rg = make_rsrc(dOb, (uint32_t)N * c.ldg);
    c.rl = make_rsrc(nlse + (int64_t)bh * N, (uint32_t)N * 4);
    c.rd = make_rsrc(ndelta + (int64_t)bh * N, (uint32_t)N * 4);
    const bool q_wave = c.wave * X::PIECES < 8;
    c.rmine = q_wave ? c.rs : c.rg;
    c.ldmine = q_wave ? c.ldq : c.ldg;
#pragma unroll
    for (int i = 0; i < X::PIECES; ++i) {
        const int piece = c.wave * X::PIECES + i;
        const int r = (piece & 7) * 8 + (c.lane >> 3);
        const uint32_t chunk = (uint32_t)(((c.lane & 7) ^ xsw(r)) * 16);
        c.voff[i] = piece < 8 ? (uint32_t)r * c.ldq + chunk + (uint32_t)(hd * HD * sizeof(T))
                              : (uint32_t)r * c.ldg + chunk + (uint32_t)(hd * HD * sizeof(T));
    }
    dkv2_issue<T, NW>(c, 0, 0);
    dkv2_issue<T, NW>(c, c.nt > 1 ? 1 : 0, 1);
    dkv2_issue<T, NW>(c, c.nt > 2 ? 2 : c.nt - 1, 2);

    // query 0 (CLS) folded in on the VALU: P = exp2(q0 . k - L0), dS = P (dO0 . v - delta0)
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
        float spart = 0.f, ppart = 0.f;
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                spart += (float)q0[s][j] * (float)k.kf[kb][s][j];
                ppart += (float)g0[s][j] * (float)k.vf[kb][s][j];
            }
        const float p0 = __builtin_amdgcn_exp2f(xhalf_sum(spart) - L0);
        const float ds0 = p0 * (xhalf_sum(ppart) - d0) * DsScale<T>::v;
        // the fold's weight (both half-waves store the same value; a guarded store here made the
        // compiler spill in the main loop)
        ((float*)(smem + 4 * X::SLOT))[c.wave * 64 + kb * 32 + c.l32] = kok[kb] ? ds0 : 0.f;
#pragma unroll
        for (int db = 0; db < 2; ++db)
#pragma unroll
            for (int g = 0; g < 4; ++g)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    k.dv[kb][db][4 * g + e] = p0 * (float)g0d[db][g][e];
                    k.dk[kb][db][4 * g + e] = ds0 * (float)q0d[db][g][e];
                }
#pragma unroll
        for (int s = 0; s < 4; ++s) frag_ds_scale<T>(k.vf[kb][s]);  // dP chains give DsScale dP
    }

    wait_vmcnt<2 * (X::PIECES + 1)>();  // slice 0 landed (slices 1, 2 in flight)
    __builtin_amdgcn_s_barrier();
    frag qa[4], ga[4];
    f32x16 S0, P0;
    load_qg<T>(qa, ga, smem, 0, c.l32, c.h);
    seeds(S0, P0, smem, 0, c.h);
    int t = 0;  // unrolled by four, then up to three single steps (see attn_bwd_dq2_kernel)
    for (; t + 4 <= c.nt; t += 4) {
        step6<T, 0>(c, k, t, qa, ga, S0, P0);
        step6<T, 1>(c, k, t + 1, qa, ga, S0, P0);
        step6<T, 2>(c, k, t + 2, qa, ga, S0, P0);
        step6<T, 3>(c, k, t + 3, qa, ga, S0, P0);
    }
    if (t < c.nt) step6<T, 0>(c, k, t++, qa, ga, S0, P0);
    if (t < c.nt) step6<T, 1>(c, k, t++, qa, ga, S0, P0);
    if (t < c.nt) step6<T, 2>(c, k, t++, qa, ga, S0, P0);
    wait_vmcnt<0>();
    if (r0q != nullptr) {
        // CLS-row fold: this block's share of query 0's dQ_0 += dS_0 k (DsScale-scaled), one
        // partial per workgroup (attn_frag.h); before the dK / dV stores, so that the K fragments
        // are dead by then
        // (the lane index is recomputed here: one more VGPR live across the loop spilled)
        __syncthreads();  // every wave is done with the ring
        const int lane = __lane_id();
        char* img = smem + c.wave * 64 * 128;
        r0_put<T>(img, k.kf[0], lane & 31, lane >> 5);
        r0_put<T>(img, k.kf[1], 32 + (lane & 31), lane >> 5);
        const float aq = r0_colsum<T, 64>(img, (const float*)(smem + 4 * X::SLOT) + c.wave * 64, lane);
        float* part = (float*)(smem + NW * 64 * 128);
        part[c.wave * 64 + lane] = aq;
        __syncthreads();
        if (c.wave == 0) {
            float sum = 0.f;
#pragma unroll
            for (int w = 0; w < NW; ++w) sum += part[w * 64 + lane];
            r0q[((int64_t)bh * nkb + kblk) * 64 + lane] = sum;
        }
    }
    // the last asm MFMAs' AGPR results: >= 18 wait states before anything reads them
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3"
                 : "+a"(k.dk[0][0]), "+a"(k.dk[0][1]), "+a"(k.dk[1][0]), "+a"(k.dk[1][1]), "+a"(k.dv[0][0]),
                   "+a"(k.dv[0][1]), "+a"(k.dv[1][0]), "+a"(k.dv[1][1]));
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
        if (kok[kb]) {  // both half-waves of a key agree
            T* rk = dqkv + ((int64_t)b * N + key[kb]) * ld + C + hd * HD;
            store_row_t21<T>(rk, k.dk[kb], dk_scale / DsScale<T>::v, c.h);
            store_row_t21<T>(rk + C, k.dv[kb], 1.0f, c.h);
        }
    }
}

}  // namespace

// launched by attention.hip's bwd2_launch (DCLIP_OPT_ATTN_BWD_BLOCK selects it); key 0 is the
// fold merge's (attn_bwd_row0_fold_merge), which also takes the dQ_0 partials written to r0q
void attn_bwd_dkdv6_launch(int dt, const void* qkv, const void* dout, const float* lse, const float* delta,
                           const float* nlse, const float* ndelta, void* dqkv, int B, int N, int H, float dk_scale,
                           float* r0q, hipStream_t st) {
    const int grid = B * H * ((N - 1 + 255) / 256);
    if (dt == DCLIP_BF16)
        attn_bwd_dkdv6_kernel<bf16><<<grid, 256, 0, st>>>((const bf16*)qkv, (const bf16*)dout, lse, delta, nlse, ndelta,
                                                          (bf16*)dqkv, N, H, dk_scale, r0q);
    else
        attn_bwd_dkdv6_kernel<f16><<<grid, 256, 0, st>>>((const f16*)qkv, (const f16*)dout, lse, delta, nlse, ndelta,
                                                         (f16*)dqkv, N, H, dk_scale, r0q);
}
