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
#include "dkdv_frag.h"

namespace {

// one 32-query sub-slice, four regions fenced in issue order (32 MFMAs):
//   R1  S / dP chains of block 0              (8)   | loads: gt / qt, block-1 seeds
//   R2  S / dP chains of block 1              (8)   | VALU: block 0's exp / mul / pack
//   R3  dV / dK of block 0 (asm, AGPR)        (8)   | VALU: block 1's exp / mul / pack; loads: next Q / dO
//   R4  dV / dK of block 1 (asm, AGPR)        (8)   | loads: next block-0 seeds
// S0 / P0 arrive seeded and qa / ga hold this sub-slice; both leave holding the next one (`nb`,
// `nsub`: the next sub-slice's slot and index)
// ISSUE (DCLIP_OPT_ATTN_BWD_BLOCK 8, round 6): the step's ring DMA is issued at the start of R4 (8
// bare asm MFMAs) instead of before R1
template <typename T, bool ISSUE = false>
__device__ __forceinline__ void sub6(K6<T>& k, int h, int l32, int lane, const char* base, int sub, const char* nb,
                                     int nsub, typename Mfma<T>::frag (&qa)[4], typename Mfma<T>::frag (&ga)[4],
                                     f32x16& S0, f32x16& P0, Dkv2Ctx<T, 4>* ic = nullptr, int it = 0, int islot = 0) {
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
    if constexpr (ISSUE) dkv2_issue<T, 4>(*ic, it, islot);
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
template <typename T, int Q, bool LATE = false>
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
    if constexpr (!LATE) dkv2_issue<T, 4>(c, t + 3 < c.nt ? t + 3 : c.nt - 1, (Q + 3) & 3);
    const char* cur = c.smem + Q * X::SLOT;
    const char* nxt = c.smem + ((Q + 1) & 3) * X::SLOT;
    sub6<T, LATE>(k, c.h, c.l32, c.lane, cur, 0, cur, 1, qa, ga, S0, P0, &c, t + 3 < c.nt ? t + 3 : c.nt - 1,
                  (Q + 3) & 3);
    sub6<T>(k, c.h, c.l32, c.lane, cur, 1, nxt, 0, qa, ga, S0, P0);
}

template <typename T, bool LATE = false>
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
        step6<T, 0, LATE>(c, k, t, qa, ga, S0, P0);
        step6<T, 1, LATE>(c, k, t + 1, qa, ga, S0, P0);
        step6<T, 2, LATE>(c, k, t + 2, qa, ga, S0, P0);
        step6<T, 3, LATE>(c, k, t + 3, qa, ga, S0, P0);
    }
    if (t < c.nt) step6<T, 0, LATE>(c, k, t++, qa, ga, S0, P0);
    if (t < c.nt) step6<T, 1, LATE>(c, k, t++, qa, ga, S0, P0);
    if (t < c.nt) step6<T, 2, LATE>(c, k, t++, qa, ga, S0, P0);
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

// ============================================================================ dkdv7: software-pipelined dkdv6
// attn_bwd_dkdv7_kernel (DCLIP_OPT_ATTN_BWD_BLOCK 7): dkdv6's arithmetic, bit for bit, in a schedule
// that spreads the softmax VALU over all four MFMA regions of a sub-slice.  dkdv6 puts block 0's
// VALU (16 exp + 16 mul + 16 converts, ~264 issue cycles) into R2 and block 1's into R3, each beside
// 8 MFMAs whose gaps hold ~192 issue cycles (MI355X_MICROARCH.md: an MFMA holds the SIMD's vector
// issue for 8 of its 32 cycles), while R1 and R4 carry none — so R2 / R3 overrun and R1 / R4 idle
// the VALU.  Here the VALU of a block is split into its P half (exp + P convert, "chunkP") and its
// dS half (multiply + dS convert, "chunkD"), and the sub-slices are software-pipelined, one period
// per sub-slice j:
//   X  S / dP chains block 1 (j)       | P 4..7 + D 0..3 of block 0 (j); j's transposed fragments
//   Y  dV / dK block 0 (j)       (asm) | D 4..7 of block 0, P 0..4 of block 1 (j); j+1's Q / dO
//                                        fragments and block-0 seeds
//   Z  S / dP chains block 0 (j+1)     | P 5..7 + D 0..7 of block 1 (j)
//   W  dV / dK block 1 (j)       (asm) | P 0..3 of block 0 (j+1); j+1's block-1 seeds; the ring's DMA
//                                        issue (once per step, in a region with VALU slack)
// ~130-200 issue cycles per region instead of 80 / 264 / 296 / 16.
template <typename T>
__device__ __forceinline__ void chunkP7(f32x16& S, Packs& pk, int i) {  // elements 2i, 2i+1: P = exp2(S), kept in S
    typedef T t2 __attribute__((ext_vector_type(2)));
    const float e0 = __builtin_amdgcn_exp2f(S[2 * i]);
    const float e1 = __builtin_amdgcn_exp2f(S[2 * i + 1]);
    S[2 * i] = e0;
    S[2 * i + 1] = e1;
    const t2 pp = {(T)e0, (T)e1};
    pk.p[i >> 2][i & 3] = __builtin_bit_cast(unsigned, pp);
}
template <typename T>
__device__ __forceinline__ void chunkD7(const f32x16& S, const f32x16& P, Packs& pk, int i) {  // dS = P dP'
    typedef T t2 __attribute__((ext_vector_type(2)));
    const float d0 = S[2 * i] * P[2 * i], d1 = S[2 * i + 1] * P[2 * i + 1];
    const t2 dd = {(T)d0, (T)d1};
    pk.d[i >> 2][i & 3] = __builtin_bit_cast(unsigned, dd);
}

// one sub-slice period (above).  In: qa / ga hold j's fragments, S0 / P0 = block 0's chains of j
// with its P chunks 0..3 done (k0.p[0]), S1 / P1 seeded for j.  Out: the same for j + 1 (at cn, sn).
template <typename T, bool ISSUE>
__device__ __forceinline__ void period7(Dkv2Ctx<T, 4>& c, K6<T>& k, int t_issue, int slot_issue, const char* cj,
                                        int sj, const char* cn, int sn, typename Mfma<T>::frag (&qa)[4],
                                        typename Mfma<T>::frag (&ga)[4], f32x16& S0, f32x16& P0, f32x16& S1,
                                        f32x16& P1, Packs& k0, Packs& k1) {
    typedef typename Mfma<T>::frag frag;
    frag gt[2][2], qt[2][2];
    // ---- X
    fence();
    load_t<T>(gt, qt, cj, sj, c.lane);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        S1 = Mfma<T>::mma(qa[s], k.kf[1][s], S1);
        chunkP7<T>(S0, k0, 4 + s);
        fence();
        P1 = Mfma<T>::mma(ga[s], k.vf[1][s], P1);
        chunkD7<T>(S0, P0, k0, s);
        fence();
    }
    // ---- Y
    load_qg<T>(qa, ga, cn, sn, c.l32, c.h);
    mfma_acc<T, true>(k.dv[0][0], gt[0][0], as_frag<T>(k0.p[0]));
    chunkD7<T>(S0, P0, k0, 4);
    chunkD7<T>(S0, P0, k0, 5);
    fence();
    mfma_acc<T, false>(k.dv[0][1], gt[0][1], as_frag<T>(k0.p[0]));
    chunkP7<T>(S1, k1, 0);
    fence();
    mfma_acc<T, false>(k.dv[0][0], gt[1][0], as_frag<T>(k0.p[1]));
    chunkD7<T>(S0, P0, k0, 6);
    chunkD7<T>(S0, P0, k0, 7);
    fence();
    mfma_acc<T, false>(k.dv[0][1], gt[1][1], as_frag<T>(k0.p[1]));
    chunkP7<T>(S1, k1, 1);
    fence();
    mfma_acc<T, false>(k.dk[0][0], qt[0][0], as_frag<T>(k0.d[0]));
    chunkP7<T>(S1, k1, 2);
    fence();
    mfma_acc<T, false>(k.dk[0][1], qt[0][1], as_frag<T>(k0.d[0]));
    chunkP7<T>(S1, k1, 3);
    fence();
    mfma_acc<T, false>(k.dk[0][0], qt[1][0], as_frag<T>(k0.d[1]));
    chunkP7<T>(S1, k1, 4);
    seeds(S0, P0, cn, sn, c.h);
    fence();
    mfma_acc<T, false>(k.dk[0][1], qt[1][1], as_frag<T>(k0.d[1]));
    fence();
    // ---- Z
    S0 = Mfma<T>::mma(qa[0], k.kf[0][0], S0);
    chunkP7<T>(S1, k1, 5);
    chunkD7<T>(S1, P1, k1, 0);
    fence();
    P0 = Mfma<T>::mma(ga[0], k.vf[0][0], P0);
    chunkP7<T>(S1, k1, 6);
    chunkD7<T>(S1, P1, k1, 1);
    fence();
    S0 = Mfma<T>::mma(qa[1], k.kf[0][1], S0);
    chunkP7<T>(S1, k1, 7);
    chunkD7<T>(S1, P1, k1, 2);
    fence();
    P0 = Mfma<T>::mma(ga[1], k.vf[0][1], P0);
    chunkD7<T>(S1, P1, k1, 3);
    fence();
    S0 = Mfma<T>::mma(qa[2], k.kf[0][2], S0);
    chunkD7<T>(S1, P1, k1, 4);
    fence();
    P0 = Mfma<T>::mma(ga[2], k.vf[0][2], P0);
    chunkD7<T>(S1, P1, k1, 5);
    fence();
    S0 = Mfma<T>::mma(qa[3], k.kf[0][3], S0);
    chunkD7<T>(S1, P1, k1, 6);
    fence();
    P0 = Mfma<T>::mma(ga[3], k.vf[0][3], P0);
    chunkD7<T>(S1, P1, k1, 7);
    fence();
    // ---- W
    if constexpr (ISSUE) dkv2_issue<T, 4>(c, t_issue, slot_issue);
    mfma_acc<T, true>(k.dv[1][0], gt[0][0], as_frag<T>(k1.p[0]));
    chunkP7<T>(S0, k0, 0);
    fence();
    mfma_acc<T, false>(k.dv[1][1], gt[0][1], as_frag<T>(k1.p[0]));
    chunkP7<T>(S0, k0, 1);
    fence();
    mfma_acc<T, false>(k.dv[1][0], gt[1][0], as_frag<T>(k1.p[1]));
    chunkP7<T>(S0, k0, 2);
    fence();
    mfma_acc<T, false>(k.dv[1][1], gt[1][1], as_frag<T>(k1.p[1]));
    chunkP7<T>(S0, k0, 3);
    fence();
    mfma_acc<T, false>(k.dk[1][0], qt[0][0], as_frag<T>(k1.d[0]));
    mfma_acc<T, false>(k.dk[1][1], qt[0][1], as_frag<T>(k1.d[0]));
    mfma_acc<T, false>(k.dk[1][0], qt[1][0], as_frag<T>(k1.d[1]));
    mfma_acc<T, false>(k.dk[1][1], qt[1][1], as_frag<T>(k1.d[1]));
    seeds(S1, P1, cn, sn, c.h);
    fence();
}

// one 64-query slice t (slot Q): the ring's wait + barrier, then its two sub-slice periods; the
// second one's Z region already runs the next slice's first block-0 chains (slot Q + 1, landed by
// this step's wait), and the DMA of slice t + 3 is issued in the first period's W
template <typename T, int Q>
__device__ __forceinline__ void step7(Dkv2Ctx<T, 4>& c, K6<T>& k, int t, typename Mfma<T>::frag (&qa)[4],
                                      typename Mfma<T>::frag (&ga)[4], f32x16& S0, f32x16& P0, f32x16& S1,
                                      f32x16& P1, Packs& k0, Packs& k1) {
    typedef Dkv2Ctx<T, 4> X;
    wait_vmcnt<X::PIECES + 1>();    // own pieces of slice t+1 landed (slice t+2 in flight)
    __builtin_amdgcn_s_barrier();  // everyone's; everyone done with slice t-1's slot
    const char* cur = c.smem + Q * X::SLOT;
    const char* nxt = c.smem + ((Q + 1) & 3) * X::SLOT;
    period7<T, true>(c, k, t + 3 < c.nt ? t + 3 : c.nt - 1, (Q + 3) & 3, cur, 0, cur, 1, qa, ga, S0, P0, S1, P1,
                     k0, k1);
    period7<T, false>(c, k, 0, 0, cur, 1, nxt, 0, qa, ga, S0, P0, S1, P1, k0, k1);
}

template <typename T>
__global__ __launch_bounds__(256, 1) void attn_bwd_dkdv7_kernel(const T* __restrict__ qkv, const T* __restrict__ dout,
                                                                const float* __restrict__ lse,
                                                                const float* __restrict__ delta,
                                                                const float* __restrict__ nlse,
                                                                const float* __restrict__ ndelta,
                                                                T* __restrict__ dqkv, int N, int H, float dk_scale,
                                                                float* __restrict__ r0q) {
    constexpr int NW = 4, KB = 64 * NW;
    typedef Dkv2Ctx<T, NW> X;
    typedef typename Mfma<T>::frag frag;
    __shared__ __attribute__((aligned(16))) char smem[4 * X::SLOT + KB * 4];
    X c;
    K6<T> k;
    c.smem = smem;
    c.lane = threadIdx.x & 63;
    c.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    c.h = c.lane >> 5;
    c.l32 = c.lane & 31;
    const int nkb = (N - 1 + KB - 1) / KB;
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
        kok[kb] = key[kb] < N;
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
    t4 q0d[2][4], g0d[2][4];
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

    // query 0 (CLS) folded in on the VALU (dkdv6)
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
        for (int s = 0; s < 4; ++s) frag_ds_scale<T>(k.vf[kb][s]);
    }

    wait_vmcnt<2 * (X::PIECES + 1)>();  // slice 0 landed (slices 1, 2 in flight)
    __builtin_amdgcn_s_barrier();
    // the pipeline's fill: block 0's chains of sub-slice 0 and their P chunks 0..3
    frag qa[4], ga[4];
    f32x16 S0, P0, S1, P1;
    Packs k0, k1;
    load_qg<T>(qa, ga, smem, 0, c.l32, c.h);
    seeds(S0, P0, smem, 0, c.h);
    fence();
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        S0 = Mfma<T>::mma(qa[s], k.kf[0][s], S0);
        P0 = Mfma<T>::mma(ga[s], k.vf[0][s], P0);
    }
    seeds(S1, P1, smem, 0, c.h);
    fence();
#pragma unroll
    for (int i = 0; i < 4; ++i) chunkP7<T>(S0, k0, i);
    fence();
    int t = 0;  // unrolled by four, then up to three single steps (slot immediates)
    for (; t + 4 <= c.nt; t += 4) {
        step7<T, 0>(c, k, t, qa, ga, S0, P0, S1, P1, k0, k1);
        step7<T, 1>(c, k, t + 1, qa, ga, S0, P0, S1, P1, k0, k1);
        step7<T, 2>(c, k, t + 2, qa, ga, S0, P0, S1, P1, k0, k1);
        step7<T, 3>(c, k, t + 3, qa, ga, S0, P0, S1, P1, k0, k1);
    }
    if (t < c.nt) step7<T, 0>(c, k, t++, qa, ga, S0, P0, S1, P1, k0, k1);
    if (t < c.nt) step7<T, 1>(c, k, t++, qa, ga, S0, P0, S1, P1, k0, k1);
    if (t < c.nt) step7<T, 2>(c, k, t++, qa, ga, S0, P0, S1, P1, k0, k1);
    wait_vmcnt<0>();
    if (r0q != nullptr) {  // the CLS-row fold (dkdv6)
        __syncthreads();
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
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3"
                 : "+a"(k.dk[0][0]), "+a"(k.dk[0][1]), "+a"(k.dk[1][0]), "+a"(k.dk[1][1]), "+a"(k.dv[0][0]),
                   "+a"(k.dv[0][1]), "+a"(k.dv[1][0]), "+a"(k.dv[1][1]));
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
        if (kok[kb]) {
            T* rk = dqkv + ((int64_t)b * N + key[kb]) * ld + C + hd * HD;
            store_row_t21<T>(rk, k.dk[kb], dk_scale / DsScale<T>::v, c.h);
            store_row_t21<T>(rk + C, k.dv[kb], 1.0f, c.h);
        }
    }
}

// ============================================================================ fp8 dK / dV (configs[4])
// attn_bwd_dkdv8_kernel: dkdv6's pass with dV^T += dO^T P and dK^T += Q^T dS on the block-scaled
// e4m3 MFMA v_mfma_scale_f32_32x32x64_f8f6f4 (twice the bf16 rate: one instruction covers a whole
// 64-query slice, K = 64), S and dP kept on the 16-bit MFMA (round 4: an e4m3 score error becomes a
// multiplicative error in P).  Operands (the hardware map of attention_fp8.hip's header: lane (r, h)
// holds 32 bytes of row r of A / column r of B, byte j is K index 16 h + 32 (j >> 4) + (j & 15), the
// K blocks 0-31 / 32-63 scaled by lanes r / r + 32):
//   B = P / dS of the lane's key, straight from the two sub-slices' S^T accumulators: byte j =
//       16 sub + reg, i.e. query 32 sub + acc_row(reg, h) of the slice, so the scale blocks are the
//       two 32-query sub-slices.  P goes in as 256 P (v_cvt_scalef32_pk_fp8_f32 divides by its f32
//       scale operand: 1/256; E8M0 2^-8 in the MFMA; P <= 1 stays below the e4m3 maximum 448 and
//       the P ~ 1/N of a long sequence far above its subnormal range); dS takes an MX block scale
//       per (key, sub-slice) from the amax of its 32 values (16 per half-wave, one permlane swap)
//   A = Q^T / dO^T rows (one head dim d each) of a pre-packed e4m3 image per slice (bwd_fp8_pack_kernel:
//       row byte p holds query qperm(p), the same K order as B; one E8M0 scale per (d, sub-slice)),
//       staged with the 16-bit slice by the same LDS-DMA ring
// Per 64-query slice and wave: 32 16-bit MFMAs (S, dP) + 8 fp8 MFMAs (2 x 2 d-blocks x {dV, dK}) in
// 1536 MFMA cycles, against dkdv6's 64 16-bit MFMAs (2048 cycles).
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef short s16x2 __attribute__((ext_vector_type(2)));

constexpr int F8_IMG = 8192 + 256;                     // per slice: Q^T8 [64][64 B] | dO^T8 [64][64 B] | 64 scale dwords
constexpr int SLOT16 = 2 * 8192 + 2 * 256;            // dkdv6's slot: Q | dO | -L | -DsScale delta
// LDS: the 16-bit ring at dkdv6's stride (its slot offsets fit the 16-bit DS immediates), then a
// ring of the fp8 images (addressed from a base of its own, likewise within the immediates)
constexpr int F8_RING = 4 * SLOT16;
constexpr float PSC = 256.0f;                          // P enters the MFMA as 256 P
constexpr int E8M0_P = 127 - 8;                        // its E8M0 scale 2^-8

// query (within the 64-query slice) at row byte p of a Q^T8 / dO^T8 row: the lane half / byte the
// two-chunk row read (tile_row8) pairs with byte p, mapped through the B operand's query order
__host__ __device__ __forceinline__ int qperm(int p) {
    const int half = (p >> 4) & 1, j = 16 * (p >> 5) + (p & 15);
    const int reg = j & 15;
    return 32 * (j >> 4) + (reg & 3) + 8 * (reg >> 2) + 4 * half;
}
// 16-B chunk XOR of a 64-B row (conflict-free 16-lane groups of ds_read_b128)
__device__ __forceinline__ int sw8r(int row) { return (row >> 2) & 3; }
// 32 bytes of row `row` of a [64][64 B] image: chunks h and 2 + h
__device__ __forceinline__ i32x8 tile_row8(const char* img, int row, int h) {
    const int x = sw8r(row);
    const i32x4 a = *(const i32x4*)(img + row * 64 + ((h ^ x) << 4));
    const i32x4 b = *(const i32x4*)(img + row * 64 + (((2 + h) ^ x) << 4));
    return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}
// the largest e with amax 2^e <= 448 (the e4m3 maximum), clamped; 0 for an all-zero block
__device__ __forceinline__ int mx_e(float amax) {
    const unsigned u = __float_as_uint(amax);
    const int E = (int)((u >> 23) & 255) - 127;
    int e = 8 - E - ((u & 0x7fffff) > 0x600000 ? 1 : 0);
    e = amax > 0.f ? e : 0;
    return e < -120 ? -120 : (e > 120 ? 120 : e);
}
__device__ __forceinline__ float pow2f(int e) { return __uint_as_float((unsigned)(127 + e) << 23); }

// four f32 -> four e4m3 bytes of one dword, each divided by `inv` (a power of two).  The first
// convert writes the low word and keeps the high one, which the second then writes: its "old"
// operand is a's own register (no v_mov of a zero per dword)
__device__ __forceinline__ int cvt4_fp8(float a, float b, float c, float d, float inv) {
    s16x2 w = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(__builtin_bit_cast(s16x2, a), a, b, inv, false);
    w = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(w, c, d, inv, true);
    return __builtin_bit_cast(int, w);
}

// acc += a . b on the block-scaled e4m3 MFMA, accumulator in AGPRs; OPA selects the byte of the
// A-scale dword (B's is byte 0).  Opens with s_nop 1: b / the scales may be VALU-written just before
template <int OPA>
__device__ __forceinline__ void mfma8_acc(f32x16& acc, const i32x8& a, int sa, const i32x8& b, int sb) {
    if constexpr (OPA == 0)
        asm volatile("s_nop 1\n\tv_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel:[0,0,0] op_sel_hi:[0,0,0]"
                     : "+a"(acc) : "v"(a), "v"(b), "v"(sa), "v"(sb));
    else if constexpr (OPA == 1)
        asm volatile("s_nop 1\n\tv_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel:[1,0,0] op_sel_hi:[0,0,0]"
                     : "+a"(acc) : "v"(a), "v"(b), "v"(sa), "v"(sb));
    else if constexpr (OPA == 2)
        asm volatile("s_nop 1\n\tv_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel:[0,0,0] op_sel_hi:[1,0,0]"
                     : "+a"(acc) : "v"(a), "v"(b), "v"(sa), "v"(sb));
    else
        asm volatile("s_nop 1\n\tv_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
                     : "+a"(acc) : "v"(a), "v"(b), "v"(sa), "v"(sb));
}

// ---------------------------------------------------------------------------- pack
// grid (nt, H, B), 256 threads: slice t (queries 1 + 64 t .. 64 + 64 t, rows past N zero) of one
// head -> f8 + ((b H + h) nt + t) F8_IMG: Q^T8 | dO^T8 rows d (byte p = query qperm(p), 16-B chunks
// swizzled by sw8r(d)) and the 64 lane dwords {dO^T(d r, sub h), dO^T(d 32+r, sub h), Q^T(d r, sub h),
// Q^T(d 32+r, sub h)} of E8M0 scales (lane = 32 h + r)
template <typename T>
__global__ __launch_bounds__(256) void bwd_fp8_pack_kernel(const T* __restrict__ qkv, const T* __restrict__ dout,
                                                           uint8_t* __restrict__ f8, int N, int H, int nt) {
    __shared__ float xs[2][64][65];
    __shared__ uint32_t scw[64];
    const int t = blockIdx.x, hd = blockIdx.y, b = blockIdx.z;
    const int tid = threadIdx.x;
    const int C = H * HD;
    {
        const int x = tid >> 7, i = (tid >> 1) & 63, d0 = (tid & 1) * 32;
        const int tok = 1 + 64 * t + i;
        float v[32];
        if (tok < N) {
            const T* src = x == 0 ? qkv + ((int64_t)b * N + tok) * 3 * C + hd * HD + d0
                                  : dout + ((int64_t)b * N + tok) * C + hd * HD + d0;
#pragma unroll
            for (int c4 = 0; c4 < 4; ++c4) {
                const uint4 r = *(const uint4*)(src + 8 * c4);
                const T* e = (const T*)&r;
#pragma unroll
                for (int k = 0; k < 8; ++k) v[8 * c4 + k] = (float)e[k];
            }
        } else {
#pragma unroll
            for (int k = 0; k < 32; ++k) v[k] = 0.f;
        }
#pragma unroll
        for (int k = 0; k < 32; ++k) xs[x][i][d0 + k] = v[k];
    }
    if (tid < 64) scw[tid] = 0u;
    __syncthreads();
    {
        const int x = tid >> 7, d = (tid >> 1) & 63, blk = tid & 1;
        float v[32];
        float am = 0.f;
#pragma unroll
        for (int k = 0; k < 32; ++k) {
            v[k] = xs[x][qperm(32 * blk + k)][d];
            am = fmaxf(am, fabsf(v[k]));
        }
        const int e = mx_e(am);
        const float inv = pow2f(-e);
        i32x4 o[2];
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int w = 0; w < 4; ++w)
                o[c][w] = cvt4_fp8(v[16 * c + 4 * w], v[16 * c + 4 * w + 1], v[16 * c + 4 * w + 2],
                                   v[16 * c + 4 * w + 3], inv);
        uint8_t* img = f8 + (((int64_t)b * H + hd) * nt + t) * F8_IMG + x * 4096 + d * 64;
#pragma unroll
        for (int c = 0; c < 2; ++c) *(i32x4*)(img + (((2 * blk + c) ^ sw8r(d)) << 4)) = o[c];
        // lane 32 blk + (d & 31), byte {dO: 0 | 1, Q: 2 | 3} by the d-block
        ((uint8_t*)scw)[(32 * blk + (d & 31)) * 4 + (x == 0 ? 2 : 0) + (d >> 5)] = (uint8_t)(127 - e);
    }
    __syncthreads();
    if (tid < 64) ((uint32_t*)(f8 + (((int64_t)b * H + hd) * nt + t) * F8_IMG + 8192))[tid] = scw[tid];
}

// ---------------------------------------------------------------------------- the dK / dV pass
template <typename T>
struct Dkv8Ctx {
    Dkv2Ctx<T, 4> c;    // the 16-bit ring's sources (its voff / SLOT stride unused here)
    rsrc_t rf;          // this (image, head)'s fp8 slice images
    uint32_t hoff;      // the head's byte offset in a 16-bit row
};

// the lane id from an opaque asm statement: the DMA offsets below are recomputed at every issue
// from it (a few VALU) instead of being held in VGPRs across the loop — held, the register
// allocator spilled them, and a scratch reload before a DMA issue waits (vmcnt) for every ring
// slice still in flight
__device__ __forceinline__ int lane_opaque() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

// slice t into ring slot `slot`: dkv2_issue's 16-bit pieces + statistics, then 2 KiB of the fp8
// image per wave and 16 scale dwords per wave: 8 vmcnt entries per wave
template <typename T>
__device__ __forceinline__ void dkv8_issue(Dkv8Ctx<T>& x, int t, int slot) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef Dkv2Ctx<T, 4> X;
    Dkv2Ctx<T, 4>& c = x.c;
    char* base = c.smem + slot * SLOT16;
    char* fbase = c.smem + F8_RING + slot * F8_IMG;
    const int ln = lane_opaque();
    const int r0 = 1 + 64 * t;
    const bool ragged = t == c.nt - 1 && c.rem < 64;  // wave-uniform
    const uint32_t soff = (uint32_t)r0 * c.ldmine;
    const int part = c.wave % 2;
    const bool is_l = c.wave < 2;
    const uint32_t idx = (uint32_t)(part * X::SPW + ln);
    // piece p = 4 wave + i covers rows r = 8 (p & 7) + ln / 8 of the slice; with those bits
    // xsw(r) = 4 ((ln >> 4) & 1) | (p & 3), so the lane part (row ln / 8, chunk (ln & 7) ^ 4 ((ln >> 4)
    // & 1)) is computed once per issue and the piece part is wave-uniform (24-bit multiplies)
    const uint32_t lrow = (uint32_t)__umul24((unsigned)(ln >> 3), c.ldmine) + x.hoff;
    const uint32_t lch = (uint32_t)((ln & 7) ^ (((ln >> 4) & 1) << 2));
    uint32_t vo[X::PIECES];
#pragma unroll
    for (int i = 0; i < X::PIECES; ++i) {
        const int p = c.wave * X::PIECES + i;
        vo[i] = lrow + (uint32_t)((p & 7) * 8) * c.ldmine + ((lch ^ (uint32_t)(p & 3)) << 4);
    }
    if (__builtin_expect(ragged, 0)) {
#pragma unroll
        for (int i = 0; i < X::PIECES; ++i) {
            const bool ok = ((c.wave * X::PIECES + i) & 7) * 8 + (ln >> 3) < c.rem;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(c.rmine, LDS_PTR(base + (c.wave * X::PIECES + i) * 1024), 16,
                                                     ok ? vo[i] + soff : 0xFFFFFFF0u, 0, 0, 0);
        }
        if (ln < X::SPW)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(is_l ? c.rl : c.rd,
                                                     LDS_PTR(base + 16384 + (is_l ? 0 : 256) + part * X::SPW * 4), 4,
                                                     (int)idx < c.rem ? (idx + (uint32_t)r0) * 4 : 0xFFFFFFF0u, 0, 0, 0);
    } else {
#pragma unroll
        for (int i = 0; i < X::PIECES; ++i)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(c.rmine, LDS_PTR(base + (c.wave * X::PIECES + i) * 1024), 16,
                                                     vo[i], soff, 0, 0);
        if (ln < X::SPW)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(is_l ? c.rl : c.rd,
                                                     LDS_PTR(base + 16384 + (is_l ? 0 : 256) + part * X::SPW * 4), 4,
                                                     idx * 4, (uint32_t)r0 * 4, 0, 0);
    }
    // the fp8 image (always whole: the pack zero-fills a ragged last slice)
    const uint32_t fo = (uint32_t)t * F8_IMG;
    const uint32_t lo = (uint32_t)(c.wave * 2048 + ln * 16);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(x.rf, LDS_PTR(fbase + c.wave * 2048), 16, lo, fo, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(x.rf, LDS_PTR(fbase + c.wave * 2048 + 1024), 16, lo + 1024, fo, 0, 0);
    if (ln < 16)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(x.rf, LDS_PTR(fbase + 8192 + c.wave * 64), 4,
                                                 (uint32_t)(8192 + c.wave * 64 + ln * 4), fo, 0, 0);
#endif
}

struct Pk8 {
    i32x8 p[2], d[2];  // [block] the e4m3 B operands: 256 P, 2^e dS (byte 16 sub + reg)
    int e[2][2];       // [block][sub] the dS block exponents
};

// elements 2i, 2i + 1 of a block's sub-slice: P' = exp2(S) kept in S, dS = P' dP' into P
__device__ __forceinline__ void fin8_chunk(f32x16& S, f32x16& P, int i) {
    const float e0 = __builtin_amdgcn_exp2f(S[2 * i]);
    const float e1 = __builtin_amdgcn_exp2f(S[2 * i + 1]);
    P[2 * i] *= e0;
    P[2 * i + 1] *= e1;
    S[2 * i] = e0;
    S[2 * i + 1] = e1;
}
// after chunks 2g, 2g + 1: the four P values of register group g into the B operand
template <int SUB>
__device__ __forceinline__ void fin8_packp(const f32x16& S, Pk8& pk, int kb, int g) {
    pk.p[kb][4 * SUB + g] = cvt4_fp8(S[4 * g], S[4 * g + 1], S[4 * g + 2], S[4 * g + 3], 1.0f / PSC);
}
// the dS block scale (amax over the sub-slice's 32 queries of this key) and its four dwords.  The
// exponent is e = 8 - frexp_exp(amax): the block maps into [128, 256) of e4m3's range, which keeps
// every value normal and costs 3 instructions (v_frexp_exp, v_sub, v_ldexp) instead of mx_e's
// "largest e" search — e4m3's relative precision is the same at any exponent of its normal range
template <int SUB>
__device__ __forceinline__ void fin8_ds(const f32x16& P, Pk8& pk, int kb) {
    float am = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) am = fmaxf(am, fabsf(P[r]));
    am = xhalf_max(am);
    const int e = 8 - __builtin_amdgcn_frexp_expf(am);
    pk.e[kb][SUB] = e;
    const float inv = __builtin_amdgcn_ldexpf(1.0f, -e);
#pragma unroll
    for (int g = 0; g < 4; ++g) pk.d[kb][4 * SUB + g] = cvt4_fp8(P[4 * g], P[4 * g + 1], P[4 * g + 2], P[4 * g + 3], inv);
}

// S / dP chains of block kb for the sub-slice in qa / ga, with `fin` VALU work (block ob's
// chunks) between the MFMAs
template <typename T, int SUB, bool VALU>
__device__ __forceinline__ void chains8(K6<T>& k, int kb, const typename Mfma<T>::frag (&qa)[4],
                                        const typename Mfma<T>::frag (&ga)[4], f32x16& S, f32x16& P, f32x16& So,
                                        f32x16& Po, Pk8& pk, int ob) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        S = Mfma<T>::mma(qa[s], k.kf[kb][s], S);
        if constexpr (VALU) fin8_chunk(So, Po, 2 * s);
        fence();
        P = Mfma<T>::mma(ga[s], k.vf[kb][s], P);
        if constexpr (VALU) {
            fin8_chunk(So, Po, 2 * s + 1);
            fin8_packp<SUB>(So, pk, ob, s);
        }
        fence();
    }
}

// one 64-query slice: S0 / P0 arrive seeded (sub 0, block 0) and qa / ga hold sub 0; both leave
// holding the next slice's sub 0.  Every LDS operand is read one region ahead of its first MFMA
// (at one wave per SIMD nothing else hides the read): sub 1's Q / dO fragments (qb / gb) in R1,
// the e4m3 A fragments in R3 (in the registers sub 0's qa / ga held), the next slice's qa / ga in R5
//   R1  S / dP block 0, sub 0   (8)        | loads qb / gb, block-1 seeds
//   R2  S / dP block 1, sub 0   (8)        | VALU block 0 sub 0; seeds block 0 sub 1
//   R3  S / dP block 0, sub 1   (8)        | VALU block 1 sub 0; e4m3 A fragments; seeds block 1 sub 1
//   R4  S / dP block 1, sub 1   (8)        | VALU block 0 sub 1
//   R5  dV / dK block 0 (e4m3)  (4 x 64 c) | VALU block 1 sub 1; next qa / ga
//   R6  dV / dK block 1 (e4m3)  (4 x 64 c) | next seeds
template <typename T, int Q>
__device__ __forceinline__ void step8(Dkv8Ctx<T>& x, K6<T>& k, int t, typename Mfma<T>::frag (&qa)[4],
                                      typename Mfma<T>::frag (&ga)[4], f32x16& S0, f32x16& P0) {
    typedef typename Mfma<T>::frag frag;
    Dkv2Ctx<T, 4>& c = x.c;
    wait_vmcnt<8>();                // own pieces of slice t+1 landed (slice t+2 in flight)
    __builtin_amdgcn_s_barrier();  // everyone's; everyone done with step t-1
    dkv8_issue<T>(x, t + 3 < c.nt ? t + 3 : c.nt - 1, (Q + 3) & 3);
    const char* cur = c.smem + Q * SLOT16;
    const char* nxt = c.smem + ((Q + 1) & 3) * SLOT16;
    f32x16 S1, P1;
    frag qb[4], gb[4];
    Pk8 pk;
    // ---- R1
    fence();
    chains8<T, 0, false>(k, 0, qa, ga, S0, P0, S1, P1, pk, 0);
    load_qg<T>(qb, gb, cur, 1, c.l32, c.h);
    seeds(S1, P1, cur, 0, c.h);
    fence();
    // ---- R2
    chains8<T, 0, true>(k, 1, qa, ga, S1, P1, S0, P0, pk, 0);
    fin8_ds<0>(P0, pk, 0);
    seeds(S0, P0, cur, 1, c.h);
    fence();
    // ---- R3
    chains8<T, 0, true>(k, 0, qb, gb, S0, P0, S1, P1, pk, 1);
    fin8_ds<0>(P1, pk, 1);
    const char* f8 = c.smem + F8_RING + Q * F8_IMG;
    const int scw = *(const int*)(f8 + 8192 + c.lane * 4);
    const i32x8 g0 = tile_row8(f8 + 4096, c.l32, c.h), g1 = tile_row8(f8 + 4096, 32 + c.l32, c.h);
    const i32x8 q0 = tile_row8(f8, c.l32, c.h), q1 = tile_row8(f8, 32 + c.l32, c.h);
    seeds(S1, P1, cur, 1, c.h);
    fence();
    // ---- R4
    chains8<T, 1, true>(k, 1, qb, gb, S1, P1, S0, P0, pk, 0);
    fin8_ds<1>(P0, pk, 0);
    fence();
    // ---- R5
    const int sd0 = 127 - (c.h ? pk.e[0][1] : pk.e[0][0]);
    mfma8_acc<0>(k.dv[0][0], g0, scw, pk.p[0], E8M0_P);
    fin8_chunk(S1, P1, 0);
    fin8_chunk(S1, P1, 1);
    fin8_packp<1>(S1, pk, 1, 0);
    fin8_chunk(S1, P1, 2);
    fin8_chunk(S1, P1, 3);
    fin8_packp<1>(S1, pk, 1, 1);
    fence();
    mfma8_acc<1>(k.dv[0][1], g1, scw, pk.p[0], E8M0_P);
    fin8_chunk(S1, P1, 4);
    fin8_chunk(S1, P1, 5);
    fin8_packp<1>(S1, pk, 1, 2);
    fin8_chunk(S1, P1, 6);
    fin8_chunk(S1, P1, 7);
    fin8_packp<1>(S1, pk, 1, 3);
    fence();
    mfma8_acc<2>(k.dk[0][0], q0, scw, pk.d[0], sd0);
    fin8_ds<1>(P1, pk, 1);
    fence();
    mfma8_acc<3>(k.dk[0][1], q1, scw, pk.d[0], sd0);
    const int sd1 = 127 - (c.h ? pk.e[1][1] : pk.e[1][0]);
    load_qg<T>(qa, ga, nxt, 0, c.l32, c.h);
    fence();
    // ---- R6
    mfma8_acc<0>(k.dv[1][0], g0, scw, pk.p[1], E8M0_P);
    mfma8_acc<1>(k.dv[1][1], g1, scw, pk.p[1], E8M0_P);
    mfma8_acc<2>(k.dk[1][0], q0, scw, pk.d[1], sd1);
    mfma8_acc<3>(k.dk[1][1], q1, scw, pk.d[1], sd1);
    seeds(S0, P0, nxt, 0, c.h);
    fence();
}

template <typename T>
__global__ __launch_bounds__(256, 1) void attn_bwd_dkdv8_kernel(const T* __restrict__ qkv, const T* __restrict__ dout,
                                                                const float* __restrict__ lse,
                                                                const float* __restrict__ delta,
                                                                const float* __restrict__ nlse,
                                                                const float* __restrict__ ndelta,
                                                                const uint8_t* __restrict__ f8, T* __restrict__ dqkv,
                                                                int N, int H, float dk_scale, float* __restrict__ r0q) {
    constexpr int NW = 4, KB = 64 * NW;
    typedef Dkv2Ctx<T, NW> X;
    typedef typename Mfma<T>::frag frag;
    __shared__ __attribute__((aligned(16))) char smem[F8_RING + 4 * F8_IMG + KB * 4];
    Dkv8Ctx<T> x;
    X& c = x.c;
    K6<T> k;
    c.smem = smem;
    c.lane = threadIdx.x & 63;
    c.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    c.h = c.lane >> 5;
    c.l32 = c.lane & 31;
    const int nkb = (N - 1 + KB - 1) / KB;
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
        kok[kb] = key[kb] < N;
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
    t4 q0d[2][4], g0d[2][4];
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
    x.rf = make_rsrc(f8 + (int64_t)bh * c.nt * F8_IMG, (uint32_t)c.nt * F8_IMG);
    x.hoff = (uint32_t)(hd * HD * sizeof(T));
    const bool q_wave = c.wave * X::PIECES < 8;
    c.rmine = q_wave ? c.rs : c.rg;
    c.ldmine = q_wave ? c.ldq : c.ldg;
    dkv8_issue<T>(x, 0, 0);
    dkv8_issue<T>(x, c.nt > 1 ? 1 : 0, 1);
    dkv8_issue<T>(x, c.nt > 2 ? 2 : c.nt - 1, 2);

    // query 0 (CLS) folded in on the VALU, as dkdv6 (the MX scales dequantise the fp8 products exactly,
    // so the accumulators hold P dO and DsScale dS q' as dkdv6's do)
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
        ((float*)(smem + F8_RING + 4 * F8_IMG))[c.wave * 64 + kb * 32 + c.l32] = kok[kb] ? ds0 : 0.f;
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
        for (int s = 0; s < 4; ++s) frag_ds_scale<T>(k.vf[kb][s]);
    }

    wait_vmcnt<16>();  // slice 0 landed (slices 1, 2 in flight)
    __builtin_amdgcn_s_barrier();
    frag qa[4], ga[4];
    f32x16 S0, P0;
    load_qg<T>(qa, ga, smem, 0, c.l32, c.h);
    seeds(S0, P0, smem, 0, c.h);
    int t = 0;
    for (; t + 4 <= c.nt; t += 4) {
        step8<T, 0>(x, k, t, qa, ga, S0, P0);
        step8<T, 1>(x, k, t + 1, qa, ga, S0, P0);
        step8<T, 2>(x, k, t + 2, qa, ga, S0, P0);
        step8<T, 3>(x, k, t + 3, qa, ga, S0, P0);
    }
    if (t < c.nt) step8<T, 0>(x, k, t++, qa, ga, S0, P0);
    if (t < c.nt) step8<T, 1>(x, k, t++, qa, ga, S0, P0);
    if (t < c.nt) step8<T, 2>(x, k, t++, qa, ga, S0, P0);
    wait_vmcnt<0>();
    if (r0q != nullptr) {  // the CLS-row fold, as dkdv6
        __syncthreads();
        const int lane = __lane_id();
        char* img = smem + c.wave * 64 * 128;
        r0_put<T>(img, k.kf[0], lane & 31, lane >> 5);
        r0_put<T>(img, k.kf[1], 32 + (lane & 31), lane >> 5);
        const float aq = r0_colsum<T, 64>(img, (const float*)(smem + F8_RING + 4 * F8_IMG) + c.wave * 64, lane);
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
    // the last (16-pass) asm MFMAs' AGPR results: a wide s_nop ladder before anything reads them
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7"
                 : "+a"(k.dk[0][0]), "+a"(k.dk[0][1]), "+a"(k.dk[1][0]), "+a"(k.dk[1][1]), "+a"(k.dv[0][0]),
                   "+a"(k.dv[0][1]), "+a"(k.dv[1][0]), "+a"(k.dv[1][1]));
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
        if (kok[kb]) {
            T* rk = dqkv + ((int64_t)b * N + key[kb]) * ld + C + hd * HD;
            store_row_t21<T>(rk, k.dk[kb], dk_scale / DsScale<T>::v, c.h);
            store_row_t21<T>(rk + C, k.dv[kb], 1.0f, c.h);
        }
    }
}

}  // namespace

// the software-pipelined form (DCLIP_OPT_ATTN_BWD_BLOCK 7), same contract as attn_bwd_dkdv6_launch
void attn_bwd_dkdv7_launch(int dt, const void* qkv, const void* dout, const float* lse, const float* delta,
                           const float* nlse, const float* ndelta, void* dqkv, int B, int N, int H, float dk_scale,
                           float* r0q, hipStream_t st) {
    const int grid = B * H * ((N - 1 + 255) / 256);
    if (dt == DCLIP_BF16)
        attn_bwd_dkdv7_kernel<bf16><<<grid, 256, 0, st>>>((const bf16*)qkv, (const bf16*)dout, lse, delta, nlse, ndelta,
                                                          (bf16*)dqkv, N, H, dk_scale, r0q);
    else
        attn_bwd_dkdv7_kernel<f16><<<grid, 256, 0, st>>>((const f16*)qkv, (const f16*)dout, lse, delta, nlse, ndelta,
                                                         (f16*)dqkv, N, H, dk_scale, r0q);
}

// launched by attention.hip's bwd2_launch (DCLIP_OPT_ATTN_BWD_BLOCK selects it); key 0 is the
// fold merge's (attn_bwd_row0_fold_merge), which also takes the dQ_0 partials written to r0q
void attn_bwd_dkdv6_launch(int dt, const void* qkv, const void* dout, const float* lse, const float* delta,
                           const float* nlse, const float* ndelta, void* dqkv, int B, int N, int H, float dk_scale,
                           float* r0q, hipStream_t st) {
    const int grid = B * H * ((N - 1 + 255) / 256);
    const bool late = dclip_option(DCLIP_OPT_ATTN_BWD_BLOCK) == 8;  // the DMA issue inside R4
#define DKDV6(TT, L)                                                                                           \
    attn_bwd_dkdv6_kernel<TT, L><<<grid, 256, 0, st>>>((const TT*)qkv, (const TT*)dout, lse, delta, nlse, ndelta, \
                                                       (TT*)dqkv, N, H, dk_scale, r0q)
    if (dt == DCLIP_BF16) {
        if (late) DKDV6(bf16, true);
        else DKDV6(bf16, false);
    } else {
        if (late) DKDV6(f16, true);
        else DKDV6(f16, false);
    }
#undef DKDV6
}

// the fp8 dK / dV pass (configs[4]): the pack of the slices' Q^T / dO^T e4m3 images into f8ws
// (attn_bwd_fp8_ws_bytes), then attn_bwd_dkdv8_kernel; the rest of the backward as dkdv6's
int64_t attn_bwd_fp8_ws_bytes(int B, int N, int H) { return (int64_t)B * H * ((N - 1 + 63) / 64) * F8_IMG; }

void attn_bwd_dkdv8_launch(int dt, const void* qkv, const void* dout, const float* lse, const float* delta,
                           const float* nlse, const float* ndelta, void* dqkv, int B, int N, int H, float dk_scale,
                           float* r0q, void* f8ws, hipStream_t st) {
    const int nt = (N - 1 + 63) / 64;
    const int grid = B * H * ((N - 1 + 255) / 256);
    const dim3 gp(nt, H, B);
    if (dt == DCLIP_BF16) {
        bwd_fp8_pack_kernel<bf16><<<gp, 256, 0, st>>>((const bf16*)qkv, (const bf16*)dout, (uint8_t*)f8ws, N, H, nt);
        attn_bwd_dkdv8_kernel<bf16><<<grid, 256, 0, st>>>((const bf16*)qkv, (const bf16*)dout, lse, delta, nlse, ndelta,
                                                          (const uint8_t*)f8ws, (bf16*)dqkv, N, H, dk_scale, r0q);
    } else {
        bwd_fp8_pack_kernel<f16><<<gp, 256, 0, st>>>((const f16*)qkv, (const f16*)dout, (uint8_t*)f8ws, N, H, nt);
        attn_bwd_dkdv8_kernel<f16><<<grid, 256, 0, st>>>((const f16*)qkv, (const f16*)dout, lse, delta, nlse, ndelta,
                                                         (const uint8_t*)f8ws, (f16*)dqkv, N, H, dk_scale, r0q);
    }
}
