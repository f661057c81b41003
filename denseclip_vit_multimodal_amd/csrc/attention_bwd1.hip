// One-pass CLS-split attention backward (the default since round 6; DCLIP_OPT_ATTN_BWD_BLOCK 0 / 10, and 9
// for the unpipelined sweep attn_bwd1_kernel): dK, dV AND dQ from a single
// key-major sweep, so every P / dS element is recomputed once (two-pass: twice) and the MFMA work is
// 5 units (S, dP, dV, dK, dQ) instead of 7 (dQ pass: S, dP, dQ; dK/dV pass: S, dP, dV, dK).
//
// Replaces the backward of nn.MultiheadAttention's softmax(q k^T d^-0.5) v (reference
// seg/denseclip/models.py:275, 287-289) with the arithmetic of the two-pass path
// (attention.hip::attn_bwd_dq2_kernel + attention_dkdv6.hip::attn_bwd_dkdv6_kernel):
//   P = exp2(S - L) (log2-domain lse), dS = P (dP - delta), dV = P^T dO, dK = dS^T q', dQ = dS K.
//
// Launch sequence (attn_bwd1_launch, then attention.hip's attn_bwd_row0_fold_merge):
//   1. attn_bwd1_prep_kernel   per query: delta = rowsum(dO o O), the negated statistics the sweep
//                              seeds its S / dP chains with, key 0's dS_q0 (kept for step 3) and the
//                              key-0 column sums dK_0 / dV_0 as per-block partials (the CLS-row fold's
//                              r0kv) — the prologue / epilogue work of the dQ pass, in the same
//                              arithmetic (so dK / dV of keys 1.. equal the two-pass result bit for bit)
//   2. attn_bwd1_kernel        the sweep: dkdv6's key-major loop (4 waves x 64 keys, one wave per
//                              SIMD, AGPR dK / dV, Q / dO / statistics slices by LDS-DMA into a 4-slot
//                              ring) plus, per 64-query slice, the slice's dS^T written to an LDS image
//                              and one 32 x 32 dQ^T tile per wave summed over the workgroup's 256 keys
//                              on the MFMA (K^T from a resident LDS image of the block's keys) —
//                              stored as a 16-bit partial per (key block, query)
//   3. attn_bwd1_dq_reduce     dQ[q] = sum over key blocks of the partials, in block order, + the key-0
//                              term dS_q0 k_0 — deterministic, no atomics
//
// The dS^T image is [256 keys][64 queries] 16-bit with an 8-byte-unit XOR swizzle
// (ds_unit_swz): conflict-free for both its writers (ds_write_b64 of 4 consecutive queries of one
// key per lane, 16 keys per lane group) and its transposing readers (ds_read_b64_tr_b16).
#include "dkdv_frag.h"

namespace {

constexpr int B1_NW = 4, B1_KB = 64 * B1_NW;  // waves, keys per workgroup
typedef Dkv2Ctx<bf16, B1_NW> B1Ring;           // the ring geometry (SLOT, PIECES) is type-independent
constexpr int B1_RING = 4 * B1Ring::SLOT;
constexpr int B1_W0 = B1_RING;                 // the CLS-row fold's per-key weights dS_0 (KB floats)
constexpr int B1_SMEM = B1_W0 + B1_KB * 4;     // ring + weights (one array: the ring's LDS-DMA target)
constexpr int B1_IMG = B1_KB * 128;            // K image / dS^T image: [256 keys][64] 16-bit each
// the two images are separate __shared__ arrays: their reads provably do not alias the ring's
// in-flight LDS-DMA writes (one array holding everything made hipcc wait vmcnt(0), i.e. for the whole
// ring, before the first dS^T image read of every step)
static_assert(B1_SMEM + 2 * B1_IMG <= 160 * 1024, "LDS");

// the lane id re-read where it is used (an opaque asm: nothing derived from it is hoisted out of the
// sweep's loop, so the dS^T / K image addresses are recomputed per step instead of holding ~14 VGPRs
// across it — the loop runs at the 256-VGPR limit)
__device__ __forceinline__ int lane_now() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

// a 16-bit fragment moved into the accumulator file (the sweep's dK / dV sums use 128 of its 256
// registers): the K / V fragments are B operands of the S / dP MFMAs only (gfx950 MFMAs read A / B
// from AGPRs), so keeping them there frees 64 arch VGPRs for the dQ tile
template <typename F>
__device__ __forceinline__ F to_agpr(F v) {
    F r;
    asm volatile("" : "=a"(r) : "0"(v));
    return r;
}

// 8-byte unit XOR of row r in the dS^T image: a bijection of r & 15 (16 keys of one ds_write_b64
// lane group hit 16 distinct units), with bit 3 flipped on r bit 1 (the transposing read's four rows
// 4h + q land in four distinct 64-B bank quarters)
__device__ __forceinline__ int ds_unit_swz(int row) { return (row & 15) ^ (((row >> 1) & 1) << 3); }

// transposing read of the dS^T image (the B operand of dQ^T += K^T dS^T): element j of half h is
// key rb*32 + 16s + 8(j>>2) + 4h + (j&3) — tr_frag's k-order, so it pairs with tr_frag(K image) —
// and MFMA column (lane & 31) is query qb*32 + (lane & 31).  The swizzle depends on the row only
// through row & 15 = 4h + q (+ 8 for the upper half), so a lane's two addresses are fixed per query
// block (ds_tr_base) and (rb, s) is an immediate offset
struct DsTrBase {
    uint32_t lo, hi;
};
__device__ __forceinline__ DsTrBase ds_tr_base(int qb, int lane) {
    const int i = lane & 15, q = i >> 2, p = i & 3, g = lane >> 4, h = lane >> 5;
    const int r = 4 * h + q;
    const int unit = qb * 8 + (g & 1) * 4 + p;
    return {(uint32_t)(r * 128 + 8 * (unit ^ ds_unit_swz(r))), (uint32_t)((r + 8) * 128 + 8 * (unit ^ ds_unit_swz(r + 8)))};
}
template <typename T>
__device__ __forceinline__ typename Mfma<T>::frag trds_frag(const char* __restrict__ img, DsTrBase a, int rb, int s) {
    typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
    const int off = (rb * 32 + 16 * s) * 128;
    i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(img + a.lo + off));
    i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(img + a.hi + off));
    typedef short s8 __attribute__((ext_vector_type(8)));
    s8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(typename Mfma<T>::frag, v);
}

// the packed dS of one 32-key block (Packs::d, accumulator layout: lane = key, word j of fragment s
// = queries 16s + 8(j>>1) + 4h + 2(j&1) + {0, 1}) into the dS^T image: four 8-byte stores of four
// consecutive queries.  dsw = (key row * 128 + 8 (h ^ ds_unit_swz(row))) of block 0; block 1's rows
// are 32 further (same swizzle), i.e. + 4 KiB
__device__ __forceinline__ uint32_t ds_put_base(int wave) {
    const int lane = threadIdx.x & 63, row = wave * 64 + (lane & 31);
    return (uint32_t)(row * 128 + 8 * ((lane >> 5) ^ ds_unit_swz(row)));
}
template <int SUB, int KB>
__device__ __forceinline__ void ds_put(char* dsimg, uint32_t dsw, const unsigned (&d)[2][4]) {
    typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const uint32_t c8 = 8u * (uint32_t)(SUB * 8 + 4 * s + 2 * i);
            const u32x2 v = {d[s][2 * i], d[s][2 * i + 1]};
            *(u32x2*)(dsimg + ((dsw ^ c8) + 4096u * KB)) = v;
        }
}

// dkdv6's sub-slice (attention_dkdv6.hip::sub6, same arithmetic and region order) plus the dS^T
// image writes of both blocks in R4 (block 0's packs are complete after R2, block 1's after R3;
// R4 carries 8 bare asm MFMAs and no VALU of its own)
template <typename T, int SUB>
__device__ __forceinline__ void sub1(K6<T>& k, int h, int l32, int lane, const char* base, const char* nb, int nsub,
                                     typename Mfma<T>::frag (&qa)[4], typename Mfma<T>::frag (&ga)[4], f32x16& S0,
                                     f32x16& P0, char* dsimg, int wave) {
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
    load_t<T>(gt, qt, base, SUB, lane);
    seeds(S1, P1, base, SUB, h);
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
    const uint32_t dsw = ds_put_base(wave);
    ds_put<SUB, 0>(dsimg, dsw, k0.d);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        mfma_acc<T, true>(k.dv[1][0], gt[s][0], as_frag<T>(k1.p[s]));
        mfma_acc<T, false>(k.dv[1][1], gt[s][1], as_frag<T>(k1.p[s]));
        mfma_acc<T, false>(k.dk[1][0], qt[s][0], as_frag<T>(k1.d[s]));
        mfma_acc<T, false>(k.dk[1][1], qt[s][1], as_frag<T>(k1.d[s]));
    }
    ds_put<SUB, 1>(dsimg, dsw, k1.d);
    seeds(S0, P0, nb, nsub, h);
    fence();
}

// dQ^T tile (32 d x 32 queries) of one slice: d block w & 1, query block w >> 1, summed over the
// workgroup's 256 keys (16 MFMAs; A = K^T from the K image, B = dS^T from the dS^T image), each
// k-step's four transposing reads issued one k-step ahead of its MFMA
template <typename T>
__device__ __forceinline__ void dq_tile(f32x16& acc, const char* kimg, const char* dsimg, int qb, int db) {
    typedef typename Mfma<T>::frag frag;
    const int lane = threadIdx.x & 63;
    const DsTrBase dsb = ds_tr_base(qb, lane);
    frag a[2], b[2];
    a[0] = tr_frag<T>(kimg, 0, 0, db, lane);
    b[0] = trds_frag<T>(dsimg, dsb, 0, 0);
    acc = zero16();
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
        if (ks + 1 < 16) {
            a[(ks + 1) & 1] = tr_frag<T>(kimg, (ks + 1) >> 1, (ks + 1) & 1, db, lane);
            b[(ks + 1) & 1] = trds_frag<T>(dsimg, dsb, (ks + 1) >> 1, (ks + 1) & 1);
        }
        acc = Mfma<T>::mma(a[ks & 1], b[ks & 1], acc);
    }
}

// one 32-column half of a dQ^T tile (lane = query row; lane half h holds columns 8g + 4h .. 8g + 4h + 3,
// g = 0..3) as two 16-B buffer stores per lane (store_row_t21's permlane pairing): row `row0 + lane`
// of the workgroup's partial block, columns 32 db .. 32 db + 31
template <typename T>
__device__ __forceinline__ void store_dq_half(rsrc_t rp, uint32_t rs, uint32_t row0, int db, const f32x16& acc,
                                              float scale) {
    typedef T t2 __attribute__((ext_vector_type(2)));
    unsigned w[4][2];
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            // bf16 partials are stored unscaled (the reduction applies scale / DsScale, a power of two:
            // the same bits); fp16 ones scaled (their range)
            const float a0 = acc[4 * g + 2 * j], a1 = acc[4 * g + 2 * j + 1];
            const t2 p = std::is_same<T, bf16>::value ? t2{(T)a0, (T)a1} : t2{(T)(a0 * scale), (T)(a1 * scale)};
            w[g][j] = __builtin_bit_cast(unsigned, p);
        }
    const int lane = lane_now();
    const uint32_t vo = (uint32_t)(lane & 31) * rs + (uint32_t)(16 * (lane >> 5) + 64 * db);
    const uint32_t so = row0 * rs;
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int G = 0; G < 4; G += 2) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const auto r = __builtin_amdgcn_permlane32_swap(w[G][j], w[G + 1][j], false, false);
            w[G][j] = r[0];
            w[G + 1][j] = r[1];
        }
        const u32x4 v = {w[G][0], w[G][1], w[G + 1][0], w[G + 1][1]};
        __builtin_amdgcn_raw_buffer_store_b128(v, rp, vo + 16 * G, so, 0);
    }
}

struct B1Out {
    rsrc_t part;       // this workgroup's partials: rows = queries, rs bytes apart (the key blocks of a
    uint32_t rs;       // query are adjacent: [B*H][Np][nkb][64] T, so the reduction reads 4-KiB runs)
    int qb, db;        // this wave's dQ tile
    float sc;          // scale / DsScale
};

// one 64-query slice t in ring slot Q:
//   wait (slice t+1 landed) + barrier A (everyone done with step t-1: its ring slot and its dS^T image
//   reads); the dQ partial of slice t-1 stored (its stores are older than the DMA issued next, so
//   the counted vmcnt of the next step still retires slice t+2 first); DMA of slice t+3; the two
//   sub-slices (dK / dV as dkdv6, dS^T into the image); lgkmcnt(0) + barrier B; the slice's dQ^T tile
template <typename T, int Q>
__device__ __forceinline__ void step1(Dkv2Ctx<T, 4>& c, K6<T>& k, int t, typename Mfma<T>::frag (&qa)[4],
                                      typename Mfma<T>::frag (&ga)[4], f32x16& S0, f32x16& P0, f32x16& dq,
                                      const B1Out& out, char* kimg, char* dsimg) {
    typedef Dkv2Ctx<T, 4> X;
    wait_vmcnt<X::PIECES + 1>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");  // no LDS access moves across a barrier
    if (t > 0)  // wave-uniform
        store_dq_half<T>(out.part, out.rs, (uint32_t)(64 * (t - 1) + 1 + out.qb * 32), out.db, dq, out.sc);
    dkv2_issue<T, 4>(c, t + 3 < c.nt ? t + 3 : c.nt - 1, (Q + 3) & 3);
    const char* cur = c.smem + Q * X::SLOT;
    const char* nxt = c.smem + ((Q + 1) & 3) * X::SLOT;
    sub1<T, 0>(k, c.h, c.l32, c.lane, cur, cur, 1, qa, ga, S0, P0, dsimg, c.wave);
    sub1<T, 1>(k, c.h, c.l32, c.lane, cur, nxt, 0, qa, ga, S0, P0, dsimg, c.wave);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    fence();
    dq_tile<T>(dq, kimg, dsimg, out.qb, out.db);
    fence();
}

template <typename T>
__global__ __launch_bounds__(256, 1) void attn_bwd1_kernel(const T* __restrict__ qkv, const T* __restrict__ dout,
                                                           const float* __restrict__ lse,
                                                           const float* __restrict__ delta,
                                                           const float* __restrict__ nlse,
                                                           const float* __restrict__ ndelta, T* __restrict__ dqkv,
                                                           T* __restrict__ dqpart, int N, int H, float dk_scale,
                                                           float scale, float* __restrict__ r0q) {
    constexpr int NW = B1_NW, KB = B1_KB;
    typedef Dkv2Ctx<T, NW> X;
    typedef typename Mfma<T>::frag frag;
    static_assert(X::SLOT == B1Ring::SLOT, "ring geometry");
    __shared__ __attribute__((aligned(128))) char smem[B1_SMEM];
    __shared__ __attribute__((aligned(128))) char kimg[B1_IMG];   // K image, swz layout
    __shared__ __attribute__((aligned(128))) char dsimg[B1_IMG];  // dS^T image, ds_unit_swz layout
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
    B1Out out;
    out.rs = (uint32_t)nkb * 128;
    out.part = make_rsrc((const char*)dqpart + ((size_t)bh * (size_t)(1 + 64 * c.nt) * nkb + kblk) * 128,
                         (uint32_t)(1 + 64 * c.nt) * out.rs);
    out.qb = c.wave >> 1;
    out.db = c.wave & 1;
    out.sc = scale / DsScale<T>::v;
    int key[2];
    bool kok[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
        key[kb] = 1 + kblk * KB + c.wave * 64 + kb * 32 + c.l32;
        kok[kb] = key[kb] < N;  // keys past N compute on key N - 1, store nothing, and are zero K rows
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

    // the K image (dQ's K^T operand): this wave's 64 key rows, zero rows for keys past N
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
        const int row = c.wave * 64 + kb * 32 + c.l32;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            frag v = k.kf[kb][s];
            if (!kok[kb])
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = (T)0.f;
            *(frag*)(kimg + row * 128 + (((2 * s + c.h) ^ xsw(row)) << 4)) = v;
        }
    }

    // query 0 (CLS) folded in on the VALU, as dkdv6
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
        ((float*)(smem + B1_W0))[c.wave * 64 + kb * 32 + c.l32] = kok[kb] ? ds0 : 0.f;
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
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            k.kf[kb][s] = to_agpr(k.kf[kb][s]);
            k.vf[kb][s] = to_agpr(k.vf[kb][s]);
        }

    wait_vmcnt<2 * (X::PIECES + 1)>();  // slice 0 landed (slices 1, 2 in flight)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the K image
    __builtin_amdgcn_s_barrier();
    frag qa[4], ga[4];
    f32x16 S0, P0, dq;
    load_qg<T>(qa, ga, smem, 0, c.l32, c.h);
    seeds(S0, P0, smem, 0, c.h);
    int t = 0;
    for (; t + 4 <= c.nt; t += 4) {
        step1<T, 0>(c, k, t, qa, ga, S0, P0, dq, out, kimg, dsimg);
        step1<T, 1>(c, k, t + 1, qa, ga, S0, P0, dq, out, kimg, dsimg);
        step1<T, 2>(c, k, t + 2, qa, ga, S0, P0, dq, out, kimg, dsimg);
        step1<T, 3>(c, k, t + 3, qa, ga, S0, P0, dq, out, kimg, dsimg);
    }
    if (t < c.nt) step1<T, 0>(c, k, t++, qa, ga, S0, P0, dq, out, kimg, dsimg);
    if (t < c.nt) step1<T, 1>(c, k, t++, qa, ga, S0, P0, dq, out, kimg, dsimg);
    if (t < c.nt) step1<T, 2>(c, k, t++, qa, ga, S0, P0, dq, out, kimg, dsimg);
    // the last slice's dQ partial
    store_dq_half<T>(out.part, out.rs, (uint32_t)(64 * (c.nt - 1) + 1 + out.qb * 32), out.db, dq, out.sc);
    wait_vmcnt<0>();
    if (r0q != nullptr) {
        // CLS-row fold (dkdv6's): this block's share of dQ_0 += dS_0 k, one partial per workgroup
        __syncthreads();
        const int lane = __lane_id();
        char* img = smem + c.wave * 64 * 128;
        r0_put<T>(img, k.kf[0], lane & 31, lane >> 5);
        r0_put<T>(img, k.kf[1], 32 + (lane & 31), lane >> 5);
        const float aq = r0_colsum<T, 64>(img, (const float*)(smem + B1_W0) + c.wave * 64, lane);
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

// ---------------------------------------------------------------------------- the pipelined sweep (default)
// attn_bwd1b_kernel: attn_bwd1_kernel's arithmetic (dK / dV bit for bit; dQ the same products summed
// in the same per-tile order) with the slice's dQ^T tile taken OFF its own barrier: the dS^T image is
// double-buffered and the 16 dQ MFMAs of slice t - 1 are spread over the eight regions of step t
// (two per region, operands read at the region's start, the MFMAs at its end, the tile's accumulator
// in AGPRs), beside the softmax VALU that leaves the matrix pipe idle in dkdv6.  LDS for the second
// dS^T buffer comes from a 3-slot ring (DMA one slice ahead instead of two) and from reading the S
// chains' K fragments out of the K image (4 ds_read_b128 per block) instead of holding them in 32
// VGPRs.
constexpr int B2_RING = 4 * B1Ring::SLOT;
constexpr int B2_SMEM = B2_RING + B1_KB * 4;  // ring + the CLS-row fold's weights
static_assert(B2_SMEM + 2 * B1_IMG <= 160 * 1024, "LDS");

// acc (AGPR) = x . b (FIRST: C = 0) or acc += x . b, the A operand x (a K^T fragment) held in AGPRs
template <typename T, bool FIRST>
__device__ __forceinline__ void mfma_dq(f32x16& acc, const typename Mfma<T>::frag& x, const typename Mfma<T>::frag& b) {
    if constexpr (FIRST) {
        if constexpr (std::is_same<T, bf16>::value)
            asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=a"(acc) : "a"(x), "v"(b));
        else
            asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, 0" : "=a"(acc) : "a"(x), "v"(b));
    } else {
        if constexpr (std::is_same<T, bf16>::value)
            asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "a"(x), "v"(b));
        else
            asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+a"(acc) : "a"(x), "v"(b));
    }
}

struct DqOps {
    int db;           // this wave's d block
    DsTrBase dsb;     // dS^T image read addresses (its query block)
};

// the dS^T operands of dQ k-steps KS, KS + 1 (keys 16 KS .. 16 KS + 31) of the previous slice's tile
template <typename T, int KS>
__device__ __forceinline__ void dq_load2(typename Mfma<T>::frag (&b)[2], const char* dsprev, const DqOps& d) {
#pragma unroll
    for (int j = 0; j < 2; ++j) b[j] = trds_frag<T>(dsprev, d.dsb, (KS + j) >> 1, (KS + j) & 1);
}

// k-steps KS, KS + 1: the K^T operands are the wave's resident AGPR fragments kt[KS], kt[KS + 1]
template <typename T, int KS, bool FIRST>
__device__ __forceinline__ void dq_mma2(f32x16& acc, const typename Mfma<T>::frag (&kt)[16],
                                        const typename Mfma<T>::frag (&b)[2]) {
    mfma_dq<T, FIRST>(acc, kt[KS], b[0]);
    mfma_dq<T, false>(acc, kt[KS + 1], b[1]);
}

// the dQ^T accumulator (AGPR, written by asm MFMAs) readable: >= 12 wait states after the last one
__device__ __forceinline__ void dq_settle(f32x16& dq) { asm volatile("s_nop 7\n\ts_nop 7" : "+a"(dq)); }

// load_qg (dkdv_frag.h) with the four chunk offsets of a row derived from one base by XOR: chunk
// (2s + h) ^ xsw(row) = 2s ^ (h ^ xsw(row)), so offset(s) = base ^ 32 s; the base passes through an
// opaque asm, so the four offsets are not hoisted out of the loop as four live VGPRs
template <typename T>
__device__ __forceinline__ void load_qg_x(typename Mfma<T>::frag (&qa)[4], typename Mfma<T>::frag (&ga)[4],
                                          const char* base, int sub, int l32, int h) {
    uint32_t o = (uint32_t)(l32 * 128 + 16 * (h ^ xsw(l32)));
    asm volatile("" : "+v"(o));
    const char* Qt = base + sub * 32 * 128;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        qa[s] = *(const typename Mfma<T>::frag*)(Qt + (o ^ (32u * s)));
        ga[s] = *(const typename Mfma<T>::frag*)(Qt + 8192 + (o ^ (32u * s)));
    }
}

// one 32-query sub-slice (sub6's regions and arithmetic) + this sub-slice's dS^T into buffer dscur +
// k-steps 8 SUB .. 8 SUB + 7 of the previous slice's dQ^T tile from buffer dsprev (two per region: the
// dS^T operands read at the region's start, the MFMAs at its end)
template <typename T, int SUB>
__device__ __forceinline__ void sub2(K6<T>& k, int h, int l32, int lane, int wave, const char* base, const char* nb,
                                     int nsub, typename Mfma<T>::frag (&qa)[4], typename Mfma<T>::frag (&ga)[4],
                                     f32x16& S0, f32x16& P0, f32x16& dq, const typename Mfma<T>::frag (&kt)[16],
                                     char* dscur, const char* dsprev, const DqOps& dqo, const B1Out* out = nullptr,
                                     uint32_t store_row = 0xFFFFFFFFu) {
    typedef typename Mfma<T>::frag frag;
    f32x16 S1, P1;
    frag gt[2][2], qt[2][2], dbf[2];
    Packs k0, k1;
    // ---- R1
    fence();
    dq_load2<T, 8 * SUB>(dbf, dsprev, dqo);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        S0 = Mfma<T>::mma(qa[s], k.kf[0][s], S0);
        asm volatile("" : "+a"(k.vf[0][s]));  // V fragments stay in AGPRs (MFMA B operands)
        P0 = Mfma<T>::mma(ga[s], k.vf[0][s], P0);
    }
    if constexpr (SUB == 0) {
        if (store_row != 0xFFFFFFFFu) {  // wave-uniform
            dq_settle(dq);
            store_dq_half<T>(out->part, out->rs, store_row, out->db, dq, out->sc);
        }
    }
    load_t<T>(gt, qt, base, SUB, lane);
    seeds(S1, P1, base, SUB, h);
    dq_mma2<T, 8 * SUB, SUB == 0>(dq, kt, dbf);
    fence();
    // ---- R2
    dq_load2<T, 8 * SUB + 2>(dbf, dsprev, dqo);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        S1 = Mfma<T>::mma(qa[s], k.kf[1][s], S1);
        fin_chunk<T>(S0, P0, k0, 2 * s);
        fence();
        asm volatile("" : "+a"(k.vf[1][s]));
        P1 = Mfma<T>::mma(ga[s], k.vf[1][s], P1);
        fin_chunk<T>(S0, P0, k0, 2 * s + 1);
        fence();
    }
    dq_mma2<T, 8 * SUB + 2, false>(dq, kt, dbf);
    fence();
    // ---- R3
    dq_load2<T, 8 * SUB + 4>(dbf, dsprev, dqo);
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
    load_qg_x<T>(qa, ga, nb, nsub, l32, h);
    dq_mma2<T, 8 * SUB + 4, false>(dq, kt, dbf);
    fence();
    // ---- R4
    dq_load2<T, 8 * SUB + 6>(dbf, dsprev, dqo);
    const uint32_t dsw = ds_put_base(wave);
    ds_put<SUB, 0>(dscur, dsw, k0.d);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        mfma_acc<T, true>(k.dv[1][0], gt[s][0], as_frag<T>(k1.p[s]));
        mfma_acc<T, false>(k.dv[1][1], gt[s][1], as_frag<T>(k1.p[s]));
        mfma_acc<T, false>(k.dk[1][0], qt[s][0], as_frag<T>(k1.d[s]));
        mfma_acc<T, false>(k.dk[1][1], qt[s][1], as_frag<T>(k1.d[s]));
    }
    ds_put<SUB, 1>(dscur, dsw, k1.d);
    seeds(S0, P0, nb, nsub, h);
    dq_mma2<T, 8 * SUB + 6, false>(dq, kt, dbf);
    fence();
}

// slice t in ring slot Q = t % 4, its dS^T into buffer DB = t & 1:
//   vmcnt (slice t + 1 landed, t + 2 in flight, as dkdv6) + lgkmcnt(0) + barrier (every wave's dS^T of
//   slice t - 1 written; every wave done with step t - 1, so slot (t + 3) % 4 and buffer DB are free);
//   the dQ partial of slice t - 2 (accumulated during step t - 1) stored; DMA of slice t + 3; the two
//   sub-slices, which also accumulate slice t - 1's dQ^T tile
template <typename T, int Q, int DB>
__device__ __forceinline__ void step2(Dkv2Ctx<T, 4>& c, K6<T>& k, int t, typename Mfma<T>::frag (&qa)[4],
                                      typename Mfma<T>::frag (&ga)[4], f32x16& S0, f32x16& P0, f32x16& dq,
                                      const B1Out& out, const DqOps& dqo, const typename Mfma<T>::frag (&kt)[16],
                                      char* dsimg) {
    typedef Dkv2Ctx<T, 4> X;
    wait_vmcnt<X::PIECES + 1>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    dkv2_issue<T, 4>(c, t + 3 < c.nt ? t + 3 : c.nt - 1, (Q + 3) & 3);
    const char* cur = c.smem + Q * X::SLOT;
    const char* nxt = c.smem + ((Q + 1) & 3) * X::SLOT;
    char* dscur = dsimg + DB * B1_IMG;
    const char* dsprev = dsimg + (DB ^ 1) * B1_IMG;
    // the dQ partial of slice t - 2 is stored from sub-slice 0's R1, beside its S / dP chains
    sub2<T, 0>(k, c.h, c.l32, c.lane, c.wave, cur, cur, 1, qa, ga, S0, P0, dq, kt, dscur, dsprev, dqo, &out,
               t >= 2 ? (uint32_t)(64 * (t - 2) + 1 + out.qb * 32) : 0xFFFFFFFFu);
    sub2<T, 1>(k, c.h, c.l32, c.lane, c.wave, cur, nxt, 0, qa, ga, S0, P0, dq, kt, dscur, dsprev, dqo);
}

// the last slice's dQ^T tile (no slice follows to hide it in): 16 MFMAs on the resident K^T fragments
template <typename T>
__device__ __forceinline__ void dq_tile_kt(f32x16& acc, const typename Mfma<T>::frag (&kt)[16], const char* dsimg,
                                           const DqOps& dqo) {
    typename Mfma<T>::frag b[2];
    dq_load2<T, 0>(b, dsimg, dqo);
    dq_mma2<T, 0, true>(acc, kt, b);
#pragma unroll
    for (int ks = 2; ks < 16; ks += 2) {
        switch (ks) {  // KS is a template argument
            case 2: dq_load2<T, 2>(b, dsimg, dqo); dq_mma2<T, 2, false>(acc, kt, b); break;
            case 4: dq_load2<T, 4>(b, dsimg, dqo); dq_mma2<T, 4, false>(acc, kt, b); break;
            case 6: dq_load2<T, 6>(b, dsimg, dqo); dq_mma2<T, 6, false>(acc, kt, b); break;
            case 8: dq_load2<T, 8>(b, dsimg, dqo); dq_mma2<T, 8, false>(acc, kt, b); break;
            case 10: dq_load2<T, 10>(b, dsimg, dqo); dq_mma2<T, 10, false>(acc, kt, b); break;
            case 12: dq_load2<T, 12>(b, dsimg, dqo); dq_mma2<T, 12, false>(acc, kt, b); break;
            default: dq_load2<T, 14>(b, dsimg, dqo); dq_mma2<T, 14, false>(acc, kt, b); break;
        }
    }
}

template <typename T>
__global__ __launch_bounds__(256, 1) void attn_bwd1b_kernel(const T* __restrict__ qkv, const T* __restrict__ dout,
                                                            const float* __restrict__ lse,
                                                            const float* __restrict__ delta,
                                                            const float* __restrict__ nlse,
                                                            const float* __restrict__ ndelta, T* __restrict__ dqkv,
                                                            T* __restrict__ dqpart, int N, int H, float dk_scale,
                                                            float scale, float* __restrict__ r0q) {
    constexpr int NW = B1_NW, KB = B1_KB;
    typedef Dkv2Ctx<T, NW> X;
    typedef typename Mfma<T>::frag frag;
    static_assert(X::SLOT == B1Ring::SLOT, "ring geometry");
    __shared__ __attribute__((aligned(128))) char smem[B2_SMEM];
    // two dS^T images (ds_unit_swz layout); the prologue's K image (swz layout, read once into the
    // resident K^T fragments) lives in the second, which step 1 overwrites
    __shared__ __attribute__((aligned(128))) char dsimg[2 * B1_IMG];
    char* kimg = dsimg + B1_IMG;
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
    B1Out out;
    out.rs = (uint32_t)nkb * 128;
    out.part = make_rsrc((const char*)dqpart + ((size_t)bh * (size_t)(1 + 64 * c.nt) * nkb + kblk) * 128,
                         (uint32_t)(1 + 64 * c.nt) * out.rs);
    out.qb = c.wave >> 1;
    out.db = c.wave & 1;
    out.sc = scale / DsScale<T>::v;
    DqOps dqo;
    dqo.db = out.db;
    dqo.dsb = ds_tr_base(out.qb, c.lane);
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

    // the K image: this wave's 64 key rows, zero rows for keys past N (their dK / dV are not stored and
    // their zero K^T columns add nothing to dQ)
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
        const int row = c.wave * 64 + kb * 32 + c.l32;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            frag v = k.kf[kb][s];
            if (!kok[kb])
#pragma unroll
                for (int j = 0; j < 8; ++j) v[j] = (T)0.f;
            *(frag*)(kimg + row * 128 + (((2 * s + c.h) ^ xsw(row)) << 4)) = v;
        }
    }
    // query 0 (CLS) folded in on the VALU, as dkdv6
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
        ((float*)(smem + B2_RING))[c.wave * 64 + kb * 32 + c.l32] = kok[kb] ? ds0 : 0.f;
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
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the K image
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    frag qa[4], ga[4], kt[16];
    f32x16 S0, P0, dq;
    // the wave's K^T fragments of its d block over the 256 keys (dQ's A operands), resident in AGPRs
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) kt[ks] = to_agpr(tr_frag<T>(kimg, ks >> 1, ks & 1, dqo.db, c.lane));
    load_qg<T>(qa, ga, smem, 0, c.l32, c.h);
    seeds(S0, P0, smem, 0, c.h);
    int t = 0;
    for (; t + 4 <= c.nt; t += 4) {
        step2<T, 0, 0>(c, k, t, qa, ga, S0, P0, dq, out, dqo, kt, dsimg);
        step2<T, 1, 1>(c, k, t + 1, qa, ga, S0, P0, dq, out, dqo, kt, dsimg);
        step2<T, 2, 0>(c, k, t + 2, qa, ga, S0, P0, dq, out, dqo, kt, dsimg);
        step2<T, 3, 1>(c, k, t + 3, qa, ga, S0, P0, dq, out, dqo, kt, dsimg);
    }
    if (t < c.nt) step2<T, 0, 0>(c, k, t++, qa, ga, S0, P0, dq, out, dqo, kt, dsimg);
    if (t < c.nt) step2<T, 1, 1>(c, k, t++, qa, ga, S0, P0, dq, out, dqo, kt, dsimg);
    if (t < c.nt) step2<T, 2, 0>(c, k, t++, qa, ga, S0, P0, dq, out, dqo, kt, dsimg);
    // the last two dQ partials: slice nt - 2 (accumulated during the last step) and slice nt - 1 (its
    // dS^T complete behind this barrier)
    wait_vmcnt<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (c.nt >= 2) {
        dq_settle(dq);
        store_dq_half<T>(out.part, out.rs, (uint32_t)(64 * (c.nt - 2) + 1 + out.qb * 32), out.db, dq, out.sc);
    }
    dq_tile_kt<T>(dq, kt, dsimg + ((c.nt - 1) & 1) * B1_IMG, dqo);
    dq_settle(dq);
    store_dq_half<T>(out.part, out.rs, (uint32_t)(64 * (c.nt - 1) + 1 + out.qb * 32), out.db, dq, out.sc);
    wait_vmcnt<0>();
    if (r0q != nullptr) {
        // CLS-row fold (dkdv6's)
        __syncthreads();
        const int lane = __lane_id();
        char* img = smem + c.wave * 64 * 128;
        r0_put<T>(img, k.kf[0], lane & 31, lane >> 5);
        r0_put<T>(img, k.kf[1], 32 + (lane & 31), lane >> 5);
        const float aq = r0_colsum<T, 64>(img, (const float*)(smem + B2_RING) + c.wave * 64, lane);
        float* part = (float*)(smem + NW * 64 * 128);
        part[c.wave * 64 + lane] = aq;
        __syncthreads();
        if (c.wave == 0) {
            float sum = 0.f;
#pragma unroll
            for (int v = 0; v < NW; ++v) sum += part[v * 64 + lane];
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

// ---------------------------------------------------------------------------- prep
// Per query q >= 1 (128 per workgroup, 2 lanes per query as the dQ pass's rows): delta, the negated
// statistics, dS_q0 (ds0v), and this block's share of key 0's column sums (r0kv: [dK_0 | dV_0], both
// DsScale-scaled as the dQ pass's epilogue writes them); query 0's delta by block 0.  The dot products
// follow attn_bwd_dq2_kernel's prologue term for term.
template <typename T>
__global__ __launch_bounds__(256) void attn_bwd1_prep_kernel(const T* __restrict__ qkv, const T* __restrict__ o,
                                                             const T* __restrict__ dout, const float* __restrict__ lse,
                                                             float* __restrict__ delta, float* __restrict__ nstat,
                                                             float* __restrict__ ds0v, float* __restrict__ r0kv, int N,
                                                             int H, int nqp, int head_minor) {
    typedef typename Mfma<T>::frag frag;
    constexpr int QB = 128;
    __shared__ __attribute__((aligned(16))) char smem[4 * 32 * 128 + 2 * QB * 4 + 4 * 128 * 4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, l32 = lane & 31;
    // workgroup -> (batch, head, query block): query block fastest (default), or (head_minor,
    // DCLIP_OPT_ATTN_PREP_ORDER 1) the H heads of one query block on adjacent workgroups, so the
    // 128-B head segments read at the same time are the adjacent pieces of the same token rows
    int blk, bh;
    if (head_minor) {
        const int hm = blockIdx.x % H, r = blockIdx.x / H;
        blk = r % nqp;
        bh = (r / nqp) * H + hm;
    } else {
        blk = blockIdx.x % nqp;
        bh = blockIdx.x / nqp;
    }
    const int b = bh / H, hd = bh % H;
    const int C = H * HD;
    const int64_t ld = 3 * (int64_t)C;
    const T* Bb = qkv + (int64_t)b * N * ld;
    const T* dOb = dout + (int64_t)b * N * C + hd * HD;
    const int q = 1 + blk * QB + wave * 32 + l32;
    const bool qok = q < N;
    const int qc = qok ? q : N - 1;
    frag qf[4], gf[4], of[4], k0[4], v0[4];
    const T* Orow = o + ((int64_t)b * N + qc) * C + hd * HD;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        k0[s] = *(const frag*)(Bb + C + hd * HD + (2 * s + h) * 8);
        v0[s] = *(const frag*)(Bb + 2 * C + hd * HD + (2 * s + h) * 8);
        qf[s] = *(const frag*)(Bb + (int64_t)qc * ld + hd * HD + (2 * s + h) * 8);
        gf[s] = *(const frag*)(dOb + (int64_t)qc * C + (2 * s + h) * 8);
        of[s] = *(const frag*)(Orow + (2 * s + h) * 8);
    }
    const float L = lse[(int64_t)bh * N + qc];
    float dpart = 0.f, spart = 0.f, ppart = 0.f;
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            dpart += (float)of[s][j] * (float)gf[s][j];
            spart += (float)qf[s][j] * (float)k0[s][j];
            ppart += (float)gf[s][j] * (float)v0[s][j];
        }
    const float dl = xhalf_sum(dpart);
    const float p0 = __builtin_amdgcn_exp2f(xhalf_sum(spart) - L);
    const float ds0 = p0 * (xhalf_sum(ppart) - dl) * DsScale<T>::v;
    if (h == 0 && qok) {
        delta[(int64_t)bh * N + q] = dl;
        nstat[(int64_t)bh * N + q] = -L;
        nstat[(int64_t)(gridDim.x / nqp) * N + (int64_t)bh * N + q] = -dl * DsScale<T>::v;
        ds0v[(int64_t)bh * N + q] = ds0;
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) frag_ds_scale<T>(gf[s]);
    float* w = (float*)(smem + 4 * 32 * 128);
    if (h == 0) {
        w[wave * 32 + l32] = qok ? ds0 : 0.f;
        w[QB + wave * 32 + l32] = qok ? p0 : 0.f;
    }
    char* img = smem + wave * 32 * 128;
    r0_put<T>(img, qf, l32, h);
    const float ak = r0_colsum<T, 32>(img, w + wave * 32, lane);
    asm volatile("" ::: "memory");
    r0_put<T>(img, gf, l32, h);
    const float av = r0_colsum<T, 32>(img, w + QB + wave * 32, lane);
    float* part = (float*)(smem + 4 * 32 * 128 + 2 * QB * 4);
    part[wave * 128 + lane] = ak;
    part[wave * 128 + 64 + lane] = av;
    if (blk == 0 && wave == 0) {  // delta of query 0 (attn_bwd_dq2_kernel's epilogue term)
        const int64_t r0 = (int64_t)b * N * C + hd * HD + lane;
        const float d0 = wave_sum((float)dout[r0] * (float)o[r0]);
        if (lane == 0) delta[(int64_t)bh * N] = d0;
    }
    __syncthreads();
    if (threadIdx.x < 128) {
        float sum = 0.f;
#pragma unroll
        for (int v = 0; v < 4; ++v) sum += part[v * 128 + threadIdx.x];
        r0kv[((int64_t)bh * nqp + blk) * 128 + threadIdx.x] = sum;
    }
}

// ---------------------------------------------------------------------------- dQ reduce
// dQ[q] = sum_j part_j[q] (key blocks in order) + dS_q0 k_0 scale / DsScale, queries 1..N-1; 8 lanes
// per query row (8 columns each), 32 rows per workgroup
template <typename T>
__global__ __launch_bounds__(256) void attn_bwd1_dq_reduce(const T* __restrict__ dqpart, const float* __restrict__ ds0v,
                                                           const T* __restrict__ qkv, T* __restrict__ dqkv, int N, int H,
                                                           int nkb, int nrb, float sc) {
    typedef T t8 __attribute__((ext_vector_type(8)));
    const int rb = blockIdx.x % nrb, bh = blockIdx.x / nrb, b = bh / H, hd = bh % H;
    const int q = 1 + rb * 32 + (threadIdx.x >> 3), c8 = (threadIdx.x & 7) * 8;
    if (q >= N) return;
    const int C = H * HD;
    const int64_t ld = 3 * (int64_t)C;
    const int64_t Np = 1 + 64 * (int64_t)((N - 1 + 63) / 64);
    const t8 kv = *(const t8*)(qkv + (int64_t)b * N * ld + C + hd * HD + c8);
    // bf16 partials are unscaled (store_dq_half): the key-0 term joins them unscaled and the sum is
    // scaled once (sc is a power of two, so this equals scaling every term)
    constexpr bool unscaled = std::is_same<T, bf16>::value;
    const float w = ds0v[(int64_t)bh * N + q] * (unscaled ? 1.0f : sc);
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = w * (float)kv[e];
    const T* p = dqpart + ((int64_t)bh * Np + q) * nkb * 64 + c8;  // this query's nkb partials, adjacent
    int j = 0;
    for (; j + 8 <= nkb; j += 8) {
        t8 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load((const t8*)(p + (j + u) * 64));
#pragma unroll
        for (int u = 0; u < 8; ++u)
#pragma unroll
            for (int e = 0; e < 8; ++e) acc[e] += (float)v[u][e];
    }
    for (; j < nkb; ++j) {
        const t8 v = __builtin_nontemporal_load((const t8*)(p + j * 64));
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += (float)v[e];
    }
    t8 r;
#pragma unroll
    for (int e = 0; e < 8; ++e) r[e] = (T)(unscaled ? acc[e] * sc : acc[e]);
    *(t8*)(dqkv + ((int64_t)b * N + q) * ld + hd * HD + c8) = r;
}

// the same sum (option DCLIP_OPT_ATTN_DQ_REDUCE 1): a workgroup takes 8 queries, whose partial runs
// (nkb x 128 B each, adjacent) it reads front to back — every wave-instruction 1 KiB contiguous — into
// LDS rows padded by 128 B (the two half-waves of the summing reads on different banks); then lane
// pair (query t / 32, columns 2 (t % 32) + {0, 1}) adds the key blocks in block order onto the key-0
// term, exactly as attn_bwd1_dq_reduce does, so the result is bit for bit the same
constexpr int RQ_Q = 8;          // queries per workgroup
constexpr int RQ_MAX_NKB = 56;   // LDS: 8 x (56 x 128 + 128) B = 57 KiB (under the 64-KiB dynamic default)
template <typename T>
__global__ __launch_bounds__(256) void attn_bwd1_dq_reduce_lds(const T* __restrict__ dqpart,
                                                               const float* __restrict__ ds0v,
                                                               const T* __restrict__ qkv, T* __restrict__ dqkv,
                                                               int N, int H, int nkb, int nrb, float sc) {
    typedef T t2 __attribute__((ext_vector_type(2)));
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    extern __shared__ __attribute__((aligned(16))) char rq_lds[];
    const int rb = blockIdx.x % nrb, bh = blockIdx.x / nrb, b = bh / H, hd = bh % H;
    const int q0 = 1 + rb * RQ_Q;
    const int C = H * HD;
    const int64_t ld = 3 * (int64_t)C;
    const int64_t Np = 1 + 64 * (int64_t)((N - 1 + 63) / 64);
    const int run = nkb * 128, stride = run + 128;  // bytes per query: in HBM / in LDS
    // rows q0 .. q0 + 7 < Np always (Np - 1 is a multiple of 64), so the reads need no guard
    const char* src = (const char*)(dqpart + ((int64_t)bh * Np + q0) * nkb * 64);
    const int chunks = RQ_Q * nkb * 8;  // 16-B chunks of the 8 runs
    for (int c = threadIdx.x; c < chunks; c += 256) {
        const int qi = c / (nkb * 8), w = c - qi * (nkb * 8);
        const u32x4 v = __builtin_nontemporal_load((const u32x4*)(src + (int64_t)c * 16));
        *(u32x4*)(rq_lds + qi * stride + w * 16) = v;
    }
    __syncthreads();
    const int qi = threadIdx.x >> 5, cp = threadIdx.x & 31;
    const int q = q0 + qi;
    if (q >= N) return;
    const t2 kv = *(const t2*)(qkv + (int64_t)b * N * ld + C + hd * HD + 2 * cp);
    constexpr bool unscaled = std::is_same<T, bf16>::value;
    const float w = ds0v[(int64_t)bh * N + q] * (unscaled ? 1.0f : sc);
    float a0 = w * (float)kv[0], a1 = w * (float)kv[1];
    const char* row = rq_lds + qi * stride + cp * 4;
#pragma unroll 8
    for (int j = 0; j < nkb; ++j) {
        const t2 v = *(const t2*)(row + j * 128);
        a0 += (float)v[0];
        a1 += (float)v[1];
    }
    const t2 r = {(T)(unscaled ? a0 * sc : a0), (T)(unscaled ? a1 * sc : a1)};
    *(t2*)(dqkv + ((int64_t)b * N + q) * ld + hd * HD + 2 * cp) = r;
}

template <typename T>
void bwd1_launch(const void* qkv, const void* o, const void* dout, const float* lse, float* delta, float* nstat,
                 float* ds0v, float* r0kv, int nqp, float* r0q, void* dqpart, void* dqkv, int B, int N, int H,
                 float scale, hipStream_t st) {
    const int nkb = (N - 1 + B1_KB - 1) / B1_KB;
    attn_bwd1_prep_kernel<T><<<B * H * nqp, 256, 0, st>>>((const T*)qkv, (const T*)o, (const T*)dout, lse, delta, nstat,
                                                          ds0v, r0kv, N, H, nqp,
                                                          dclip_option(DCLIP_OPT_ATTN_PREP_ORDER) == 1);
    if (dclip_option(DCLIP_OPT_ATTN_BWD_BLOCK) != 9)  // the pipelined sweep (default); 9: the barrier form
        attn_bwd1b_kernel<T><<<B * H * nkb, 256, 0, st>>>((const T*)qkv, (const T*)dout, lse, delta, nstat,
                                                          nstat + (int64_t)B * H * N, (T*)dqkv, (T*)dqpart, N, H,
                                                          1.0f / LOG2E, scale, r0q);
    else
        attn_bwd1_kernel<T><<<B * H * nkb, 256, 0, st>>>((const T*)qkv, (const T*)dout, lse, delta, nstat,
                                                         nstat + (int64_t)B * H * N, (T*)dqkv, (T*)dqpart, N, H,
                                                         1.0f / LOG2E, scale, r0q);
    if (dclip_option(DCLIP_OPT_ATTN_DQ_REDUCE) == 1 && nkb <= RQ_MAX_NKB) {
        const int nrb = (N - 1 + RQ_Q - 1) / RQ_Q;
        attn_bwd1_dq_reduce_lds<T><<<B * H * nrb, 256, RQ_Q * (nkb * 128 + 128), st>>>(
            (const T*)dqpart, ds0v, (const T*)qkv, (T*)dqkv, N, H, nkb, nrb, scale / DsScale<T>::v);
        return;
    }
    const int nrb = (N - 1 + 31) / 32;
    attn_bwd1_dq_reduce<T><<<B * H * nrb, 256, 0, st>>>((const T*)dqpart, ds0v, (const T*)qkv, (T*)dqkv, N, H, nkb, nrb,
                                                        scale / DsScale<T>::v);
}

}  // namespace

int attn_bwd1_prep_blocks(int N) { return (N - 1 + 127) / 128; }

int64_t attn_bwd1_part_bytes(int B, int N, int H) {
    const int64_t nkb = (N - 1 + B1_KB - 1) / B1_KB, np = 1 + 64 * (int64_t)((N - 1 + 63) / 64);
    return (int64_t)B * H * nkb * np * 128;
}

void attn_bwd1_launch(int dt, const void* qkv, const void* o, const void* dout, const float* lse, float* delta,
                      float* nstat, float* ds0v, float* r0kv, float* r0q, void* dqpart, void* dqkv, int B, int N,
                      int H, float scale, hipStream_t st) {
    const int nqp = attn_bwd1_prep_blocks(N);
    if (dt == DCLIP_BF16)
        bwd1_launch<bf16>(qkv, o, dout, lse, delta, nstat, ds0v, r0kv, nqp, r0q, dqpart, dqkv, B, N, H, scale, st);
    else
        bwd1_launch<f16>(qkv, o, dout, lse, delta, nstat, ds0v, r0kv, nqp, r0q, dqpart, dqkv, B, N, H, scale, st);
}
