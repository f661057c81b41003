// Fragment helpers shared by the attention kernels (attention.hip, attention_dkdv6.hip):
// the swizzled 128-B-row LDS image, MFMA operand fragments, the O^T-layout row store and the
// LDS-DMA ring of the CLS-split dK/dV passes.  Device-only inline code (each including
// translation unit gets its own copy).
#pragma once
#include "common.h"

namespace {

constexpr int HD = 64;  // head dim
constexpr float LOG2E = 1.4426950408889634f;

// chunk XOR of row r: bit 2 from row bit 1, bits 1..0 from row bits 4..3
__device__ __forceinline__ int xsw(int row) { return (((row >> 1) & 1) << 2) | ((row >> 3) & 3); }

// byte offset of 16-bit element (row, col) in a [rows][64] image
__device__ __forceinline__ int swz(int row, int col) {
    return row * 128 + (((col >> 3) ^ xsw(row)) << 4) + ((col & 7) << 1);
}

template <typename T>
__device__ __forceinline__ typename Mfma<T>::frag row_frag(const char* __restrict__ img, int row, int chunk) {
    return *(const typename Mfma<T>::frag*)(img + row * 128 + ((chunk ^ xsw(row)) << 4));
}

// A-operand fragment of X^T for a product that sums over the ROWS of an image whose
// k-order follows the "accumulator as B-operand" permutation: element j of half h is
// image row rb*32 + 16s + 8(j>>2) + 4h + (j&3), MFMA row (lane & 31) is image column
// cb*32 + (lane & 31).  Two transposing 4x16 LDS reads.
template <typename T>
__device__ __forceinline__ typename Mfma<T>::frag tr_frag(const char* __restrict__ img, int rb, int s, int cb, int lane) {
    const int i = lane & 15, q = i >> 2, p = i & 3, g = lane >> 4, h = lane >> 5;
    const int row = rb * 32 + 16 * s + 4 * h + q;
    const int col = cb * 32 + (g & 1) * 16 + 4 * p;
    typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
    i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(img + swz(row, col)));
    i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(img + swz(row + 8, col)));
    typedef short s8 __attribute__((ext_vector_type(8)));
    s8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(typename Mfma<T>::frag, v);
}

// 16-bit B-operand fragment from accumulator registers 8s..8s+7 (built from explicit
// register pairs: one v_cvt_pk per dword, no 16-bit re-alignment)
template <typename T>
__device__ __forceinline__ typename Mfma<T>::frag pack_frag(const f32x16& a, int s) {
    typedef T t2 __attribute__((ext_vector_type(2)));
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    u32x4 w;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const t2 p = {(T)a[8 * s + 2 * j], (T)a[8 * s + 2 * j + 1]};
        w[j] = __builtin_bit_cast(unsigned, p);
    }
    return __builtin_bit_cast(typename Mfma<T>::frag, w);
}

__device__ __forceinline__ f32x16 zero16() {
    f32x16 z;
#pragma unroll
    for (int e = 0; e < 16; ++e) z[e] = 0.f;
    return z;
}

__device__ __forceinline__ f32x16 splat16(float v) {
    f32x16 z;
#pragma unroll
    for (int e = 0; e < 16; ++e) z[e] = v;
    return z;
}

// dS = P (dP - delta) is ~|dO|/N in magnitude; for fp16 operands it is pre-scaled by 2^4
// before the 16-bit conversion (with dO already gradient-scaled to amax ~16 by the host,
// ops.grad_scale, this keeps N = 8193 values out of the fp16 subnormal range without
// overflow risk) and the dQ / dK accumulators are scaled back in the epilogue.  bf16 has
// the fp32 exponent range.
template <typename T> struct DsScale { static constexpr float v = 1.0f; };
template <> struct DsScale<f16> { static constexpr float v = 16.0f; };

// frag *= DsScale (a power of two: exact unless the value overflows, which the gradient scaling
// of the callers rules out).  The CLS-split backward passes apply the fp16 dS pre-scale this way,
// to the register-resident dO (dQ pass) / V (dK/dV pass) fragments once per workgroup, with the
// matching -DsScale * delta seeds, instead of one multiply per dS element.
template <typename T>
__device__ __forceinline__ void frag_ds_scale(typename Mfma<T>::frag& f) {
    if constexpr (DsScale<T>::v != 1.0f) {
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = (T)((float)f[j] * DsScale<T>::v);
    }
}

// accumulator register r -> row offset within a 32x32 tile (column = lane & 31)
__device__ __forceinline__ int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// row max / sum across the two half-waves (lanes l and l ^ 32) on the VALU
__device__ __forceinline__ float xhalf_max(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xhalf_sum(float x) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}


// 16-B stores of one output row held as the O^T accumulator layout (T21): lane h of a row
// holds columns 8G + 4h .. 8G + 4h + 3 of every 8-column group G; one permlane32 swap per
// dword pairs groups (G, G+1) into 16 contiguous bytes per lane.
template <typename T>
__device__ __forceinline__ void store_row_t21(T* row, const f32x16 (&acc)[2], float scale, int h) {
    typedef T t2 __attribute__((ext_vector_type(2)));
    unsigned w[8][2];  // group G = 4 db + g: two dwords (columns +0..1, +2..3 of this lane's half)
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const t2 p = {(T)(acc[db][4 * g + 2 * j] * scale), (T)(acc[db][4 * g + 2 * j + 1] * scale)};
                w[4 * db + g][j] = __builtin_bit_cast(unsigned, p);
            }
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int G = 0; G < 8; G += 2) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const auto r = __builtin_amdgcn_permlane32_swap(w[G][j], w[G + 1][j], false, false);
            w[G][j] = r[0];
            w[G + 1][j] = r[1];
        }
        const u32x4 v = {w[G][0], w[G][1], w[G + 1][0], w[G + 1][1]};
        *(u32x4*)((char*)row + 16 * G + 16 * h) = v;
    }
}

// ---------------------------------------------------------------------------- CLS-row fold
// The CLS row's backward sums that run over the OTHER axis of a pass — dK_0 / dV_0 (sums over
// queries) in the query-major dQ pass, dQ_0 (a sum over keys) in the key-major dK/dV pass — are
// taken in the pass's epilogue from the register-resident rows: each wave copies its rows into
// a plain [rows][64] LDS image (the ring is free by then) and lane d sums column d against the
// per-row weights the prologue parked in LDS.  One partial per workgroup goes to the workspace;
// attn_bwd_row0_fold_merge adds them up in a fixed order (deterministic, no atomics).
template <typename T>
__device__ __forceinline__ void r0_put(char* img, const typename Mfma<T>::frag (&x)[4], int row, int h) {
#pragma unroll
    for (int s = 0; s < 4; ++s) *(typename Mfma<T>::frag*)(img + row * 128 + (2 * s + h) * 16) = x[s];
}

// sum over the image's ROWS rows of w[r] * img[r][lane] (lane < 64: one column per lane).  The
// image was written by this wave's own lanes: LDS executes a wave's operations in order, the
// wait only keeps the compiler from hoisting the reads over the writes
template <typename T, int ROWS>
__device__ __forceinline__ float r0_colsum(const char* img, const float* w, int lane) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    float acc = 0.f;
#pragma unroll 8
    for (int r = 0; r < ROWS; ++r) acc += w[r] * (float)((const T*)(img + r * 128))[lane];
    return acc;
}

// ---------------------------------------------------------------------------- dK/dV pass, CLS split
// Key-major dK/dV pass on N = 1 + 32*NW*k: keys 1..N-1 in full blocks (key 0 by the row-0
// kernels above), query 0 folded into every key's dK / dV on the VALU in the prologue, and
// query slices 1 + 64t .. 64 + 64t staged by LDS-DMA — Q and dO pieces plus the slice's L and
// delta (one masked dword DMA per wave) — into a 4-slot ring three slices ahead, one bare
// barrier per slice behind a counted vmcnt.  The statistics are negated where they seed the
// S / dP accumulators.
template <typename T, int NW>
struct Dkv2Ctx {
    typedef typename Mfma<T>::frag frag;
    static constexpr int PIECES = 16 / NW;  // 1-KiB pieces of a slice (Q + dO) per wave
    static constexpr int SLOT = 2 * 8192 + 2 * 256;  // [Q | dO | L | delta]
    static constexpr int SPW = 128 / NW;             // statistics per wave per slice
    char* smem;
    rsrc_t rs, rg, rl, rd;  // qkv rows, dO rows, lse, delta of this (batch, head)
    rsrc_t rmine;           // this wave's piece source (rs for the Q waves, rg for the dO waves)
    uint32_t voff[PIECES];
    uint32_t ldq, ldg, ldmine;  // row pitches (bytes)
    int nt, lane, l32, h, wave;
    int rem;  // queries in the last slice (64 unless N - 1 is ragged)
    frag kf[4], vf[4];
    f32x16 dk[2], dv[2];
};

template <typename T, int NW>
__device__ __forceinline__ void dkv2_issue(Dkv2Ctx<T, NW>& c, int t, int slot) {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef Dkv2Ctx<T, NW> X;
    char* base = c.smem + slot * X::SLOT;
    const int r0 = 1 + 64 * t;
    // a wave's pieces are all Q (waves 0 .. NW/2-1) or all dO: its source resource and row
    // pitch were chosen once at setup, so the issue is one straight-line block (no branches
    // splitting the step's schedule).  A ragged last slice (rem < 64 queries) goes with the
    // whole offset in the voffset and the rows past N at 0xFFFFFFF0 (zeros, as in fwd2_issue):
    // a zero Q / dO row and zero statistics give dS = 0 and zero dV / dK terms.
    const bool ragged = t == c.nt - 1 && c.rem < 64;  // wave-uniform
    const uint32_t soff = (uint32_t)r0 * c.ldmine;
    const int part = c.wave % (NW / 2);
    const bool is_l = c.wave < NW / 2;
    const uint32_t idx = (uint32_t)(part * X::SPW + c.lane);  // this lane's statistic in the slice
    if (__builtin_expect(ragged, 0)) {
#pragma unroll
        for (int i = 0; i < X::PIECES; ++i) {
            const int piece = c.wave * X::PIECES + i;
            const bool ok = (piece & 7) * 8 + (c.lane >> 3) < c.rem;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(c.rmine, LDS_PTR(base + piece * 1024), 16,
                                                     ok ? c.voff[i] + soff : 0xFFFFFFF0u, 0, 0, 0);
        }
        if (c.lane < X::SPW)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(is_l ? c.rl : c.rd,
                                                     LDS_PTR(base + 16384 + (is_l ? 0 : 256) + part * X::SPW * 4), 4,
                                                     (int)idx < c.rem ? (idx + (uint32_t)r0) * 4 : 0xFFFFFFF0u, 0, 0, 0);
        return;
    }
#pragma unroll
    for (int i = 0; i < X::PIECES; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(c.rmine, LDS_PTR(base + (c.wave * X::PIECES + i) * 1024), 16,
                                                 c.voff[i], soff, 0, 0);
    // statistics: waves 0 .. NW/2-1 load L, the others delta, SPW values each
    if (c.lane < X::SPW)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(is_l ? c.rl : c.rd,
                                                 LDS_PTR(base + 16384 + (is_l ? 0 : 256) + part * X::SPW * 4), 4,
                                                 idx * 4, (uint32_t)r0 * 4, 0, 0);
#endif
}

}  // namespace
