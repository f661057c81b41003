// fp8 (OCP e4m3) attention forward — BASELINE config 5 ("fp8 MFMA attention").
//
// Same contract as dclip_attn_fwd (reference: the nn.MultiheadAttention core of
// ResidualAttentionBlock.attention, models.py:287-289; q columns of the packed qkv pre-multiplied
// by d^-0.5 * log2(e)), computed on the block-scaled gfx950 MFMA v_mfma_scale_f32_32x32x64_f8f6f4,
// which runs at twice the bf16 rate (one instruction covers K = 64: a whole head dimension, or
// 64 keys) and applies an E8M0 (power-of-two) scale per lane to each operand's 32-element K block.
//
// MX block scales.  Every 32-element K block of every operand row carries its own power-of-two
// scale, the largest 2^s with amax * 2^s <= 448 (the e4m3 maximum): q and k rows per 32-dim half,
// V^T rows (one head dim d) per 32-key half of each 64-key unit.  So no global amax pass is
// needed (each block's scale is local to the pack), small rows keep their precision, and the
// MFMA hands back S exactly dequantised and already in the log2 domain: the softmax takes
// exp2 of the accumulator as it stands — no per-score dequantisation multiply.
//
// Two launches after query 0 (the CLS row: the 16-bit forward's split-key row pass):
//   1. fp8mx_pack_kernel  tokens 1..N-1 of one 64-token unit per workgroup:
//                           q8, k8 [b][h][n1p][64] bytes (token rows), qs [b][h][n1p][2] E8M0
//                           vt8    [b][h][64][n1p] bytes (V transposed, keys permuted per unit,
//                                                       see vt_key() below)
//                           sc     [b][h][unit][64] dwords: lane (half, r)'s four E8M0 scales
//                                  {K(key r, d-half), K(key 32+r, d-half), V^T(d r, key-half),
//                                  V^T(d 32+r, key-half)}, half = the d-half / key-half
//                         rows past N are zero
//   2. attn_fp8mx_kernel  CLS-split flash forward (the 16-bit attn_fwd2_kernel's structure): key 0
//                         folded into every query's softmax state on the VALU from the 16-bit
//                         qkv; keys 1..N-1 in 64-key units staged by LDS-DMA (K tile, V^T tile,
//                         the unit's 256 scale bytes) into a 4-slot ring three units ahead; per
//                         wave and unit
//                           S^T = K Q^T     2 MFMAs, accumulators seeded with -m (the running
//                                           max), scales: K (opsel 0/1 of the lane's dword), q
//                           softmax         P = exp2(S) against the running reference; when a
//                                           lane's row sum passes 448 (the e4m3 maximum) the
//                                           reference moves to the unit's max and P is redone
//                           O^T += V^T P^T  2 MFMAs, P^T converted to e4m3 in registers, scales:
//                                           V^T (opsel 2/3), 1 for P
//
// Operand maps.  For the 32x32x64 f8f6f4 MFMA a lane (r = lane & 31, half = lane >> 5) holds
// 32 bytes of row r of A (column r of B); byte j of half `half` is the K index
// kappa_hw(half, j) = 16 half + 32 (j >> 4) + (j & 15), and the two 32-element scale blocks are
// K 0-31 (bytes 0-15 of both halves), scaled by lane r's E8M0 byte, and K 32-63 (bytes 16-31),
// scaled by lane r + 32's (measured: tools/mfma_scale_probe.hip, profiles/r03/r03k_mfma_scale_probe.log).
// For S^T = K Q^T the K index is the head dim: a lane loads 16-byte chunks `half` and 2 + half of
// its 64-byte token row, so kappa_hw is d itself and the blocks are d 0-31 / 32-63, the lane's
// scale that of d-block `half`.  For O^T = V^T P^T it is the key: the S^T accumulator of key
// sub-tile t has key (reg & 3) + 8 (reg >> 2) + 4 half in register reg, so the lane's 32 P values
// are used as bytes j = 16 t + reg, which makes byte (half, j) = key kappa(half, j) below and the
// scale blocks keys 0-31 / 32-63 of the unit (block t, scale from the lane of half t); the pack
// stores each unit's V^T row with key vt_key(q) at byte q, so that the same two-chunk row load
// (tile_row) pairs every V^T byte with its P byte, and takes the block amax over the natural key
// halves (bytes 0-31 / 32-63 of the row).
#include "attn_frag.h"

#include <type_traits>

namespace {

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

constexpr int FP8_FMT_E4M3 = 0;  // f8f6f4 format code of OCP e4m3
constexpr int E8M0_ONE = 127;    // scale 2^0
constexpr int U8SLOT = 8192 + 256;  // ring slot: K tile [64][64 B] | V^T tile [64][64 B] | 64 scale dwords

__device__ __forceinline__ int kappa(int half, int j) {  // key of P byte j of a lane of `half`
    const int t = j >> 4, reg = j & 15;
    return 32 * t + (reg & 3) + 8 * (reg >> 2) + 4 * half;
}
// key stored at byte p of a unit's V^T row: the byte a lane of half (p >> 4) & 1 loads as its
// byte 16 (p >> 5) + (p & 15) (tile_row), paired with that P byte
__device__ __forceinline__ int vt_key(int p) { return kappa((p >> 4) & 1, 16 * (p >> 5) + (p & 15)); }

// the block scale exponent: the largest s with amax * 2^s <= 448 (0 for an all-zero block)
__device__ __forceinline__ int mx_exp(float amax) {
    if (!(amax > 0.f)) return 0;
    int e;
    frexpf(448.0f / amax, &e);  // 448 / amax = f 2^e, f in [0.5, 1): floor(log2) = e - 1
    return max(-120, min(120, e - 1));
}

// 4 floats -> 4 e4m3 bytes of one dword (clamped to +-448: the convert does not saturate)
__device__ __forceinline__ int pack4_fp8(float a, float b, float c, float d) {
    a = fminf(fmaxf(a, -448.f), 448.f);
    b = fminf(fmaxf(b, -448.f), 448.f);
    c = fminf(fmaxf(c, -448.f), 448.f);
    d = fminf(fmaxf(d, -448.f), 448.f);
    int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
    return __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
}
// the same for softmax probabilities (in [0, 1]: no clamp)
__device__ __forceinline__ int pack4_fp8_unit(float a, float b, float c, float d) {
    int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
    return __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
}

template <int OPSEL_A>
__device__ __forceinline__ f32x16 mfma_mx(i32x8 a, int sa, i32x8 b, int sb, f32x16 c) {
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, FP8_FMT_E4M3, FP8_FMT_E4M3, OPSEL_A, sa, 0, sb);
}

// 16-B chunk XOR of a 64-B row in a ring tile (conflict-free 16-lane groups of ds_read_b128)
__device__ __forceinline__ int sw8(int row) { return (row >> 2) & 3; }

// ---------------------------------------------------------------------------- 1. pack
// grid (n1p / 64, H, B), 256 threads: tokens 1 + 64u .. 64 + 64u of one head
// QK = false (the default S16 kernel, which takes q and k from the 16-bit qkv): V^T only
template <typename T, bool QK>
__global__ void __launch_bounds__(256) fp8mx_pack_kernel(const T* __restrict__ qkv, uint8_t* __restrict__ q8,
                                                         uint8_t* __restrict__ qs, uint8_t* __restrict__ k8,
                                                         uint8_t* __restrict__ vt8, uint32_t* __restrict__ sc, int N,
                                                         int H, int n1p) {
    __shared__ float vs[64][65];
    __shared__ uint32_t scw[64];
    const int C = H * 64;
    const int u = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
    const int tid = threadIdx.x;
    const int64_t hb = (int64_t)b * H + h;
    if constexpr (!QK) {
        // the unit's V rows into LDS (thread -> token t, 16-dim chunk d0)
        const int t = tid >> 2, d0 = (tid & 3) * 16;
        const int tok = 1 + u * 64 + t;
        if (tok < N) {
            const T* row = qkv + ((int64_t)b * N + tok) * 3 * C + 2 * C + h * 64 + d0;
            const uint4 r0 = *(const uint4*)row, r1 = *(const uint4*)(row + 8);
            const T* e0 = (const T*)&r0;
            const T* e1 = (const T*)&r1;
#pragma unroll
            for (int i = 0; i < 8; ++i) vs[t][d0 + i] = (float)e0[i], vs[t][d0 + 8 + i] = (float)e1[i];
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) vs[t][d0 + i] = 0.f;
        }
    } else {
        // q and k rows: thread -> (token t, 16-dim chunk d0); a 32-dim block is two threads
        const int t = tid >> 2, d0 = (tid & 3) * 16, dh = d0 >> 5;
        const int tok = 1 + u * 64 + t;
        float q[16], k[16];
        if (tok < N) {
            const T* row = qkv + ((int64_t)b * N + tok) * 3 * C + h * 64 + d0;
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                const uint4 r0 = *(const uint4*)(row + p * C), r1 = *(const uint4*)(row + p * C + 8);
                const T* e0 = (const T*)&r0;
                const T* e1 = (const T*)&r1;
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const float x0 = (float)e0[i], x1 = (float)e1[i];
                    if (p == 0) q[i] = x0, q[8 + i] = x1;
                    else if (p == 1) k[i] = x0, k[8 + i] = x1;
                    else vs[t][d0 + i] = x0, vs[t][d0 + 8 + i] = x1;
                }
            }
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) q[i] = k[i] = vs[t][d0 + i] = 0.f;
        }
        float aq = 0.f, ak = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) aq = fmaxf(aq, fabsf(q[i])), ak = fmaxf(ak, fabsf(k[i]));
        aq = fmaxf(aq, __shfl_xor(aq, 1, 64));
        ak = fmaxf(ak, __shfl_xor(ak, 1, 64));
        const int sq = mx_exp(aq), sk = mx_exp(ak);
        i32x4 oq, ok;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            oq[i] = pack4_fp8(ldexpf(q[4 * i], sq), ldexpf(q[4 * i + 1], sq), ldexpf(q[4 * i + 2], sq),
                              ldexpf(q[4 * i + 3], sq));
            ok[i] = pack4_fp8(ldexpf(k[4 * i], sk), ldexpf(k[4 * i + 1], sk), ldexpf(k[4 * i + 2], sk),
                              ldexpf(k[4 * i + 3], sk));
        }
        const int64_t r = hb * n1p + u * 64 + t;
        *(i32x4*)(q8 + r * 64 + d0) = oq;
        *(i32x4*)(k8 + r * 64 + d0) = ok;
        if ((tid & 1) == 0) {
            qs[r * 2 + dh] = (uint8_t)(E8M0_ONE - sq);
            ((uint8_t*)scw)[(dh * 32 + (t & 31)) * 4 + (t >> 5)] = (uint8_t)(E8M0_ONE - sk);
        }
    }
    __syncthreads();
    {
        // V^T: thread -> (d, bytes 16p .. 16p + 15 of the unit's row, p = tid & 3), byte q holding
        // key vt_key(q): keys of half p >> 1 only, so the thread pair (p, p ^ 1) spans one scale
        // block (the unit's natural key halves)
        const int d = tid >> 2, p = tid & 3, s0 = p * 16;
        float e[16];
        float am = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            e[i] = vs[vt_key(s0 + i)][d];
            am = fmaxf(am, fabsf(e[i]));
        }
        am = fmaxf(am, __shfl_xor(am, 1, 64));
        const int kh = p >> 1;
        const int sv = mx_exp(am);
        i32x4 o;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            o[i] = pack4_fp8(ldexpf(e[4 * i], sv), ldexpf(e[4 * i + 1], sv), ldexpf(e[4 * i + 2], sv),
                             ldexpf(e[4 * i + 3], sv));
        *(i32x4*)(vt8 + (hb * 64 + d) * n1p + u * 64 + s0) = o;
        if ((p & 1) == 0) ((uint8_t*)scw)[(kh * 32 + (d & 31)) * 4 + 2 + (d >> 5)] = (uint8_t)(E8M0_ONE - sv);
    }
    __syncthreads();
    if (tid < 64) sc[(hb * (n1p / 64) + u) * 64 + tid] = scw[tid];
}

// ---------------------------------------------------------------------------- 2. attention
// S16 (the default): S^T = K Q^T on the 16-bit MFMA from the 16-bit qkv (K tiles staged by
// LDS-DMA in the 128-B-row swizzled image of the 16-bit kernels) and only O^T += V^T P^T on the
// block-scaled fp8 MFMA.  The scores are exponentiated, so an e4m3 error in S (3 mantissa bits:
// ~6 % of the score's spread) becomes a multiplicative error in P that grows with the score
// scale (27.8 % from exact on a head with 16x scores, round 3), whereas P V's e4m3 errors
// average over the keys.  Ring slot for S16: [K 16-bit 64 x 128 B | V^T 64 x 64 B | scales].
constexpr int U16SLOT = 8192 + 4096 + 256;

template <bool S16>
struct F8Ctx {
    char* smem;     // 4 ring slots of U8SLOT bytes
    rsrc_t rmine;   // this wave's piece source: the K plane (waves 0-3) or the V^T plane (4-7)
    rsrc_t rsc;     // the scale plane of this (image, head)
    uint32_t voff;  // this lane's source offset inside a tile (its 16 B of the wave's 1-KiB piece)
    uint32_t soff_unit;  // the piece's source stride per unit (4096 for K, 64 for V^T)
    int nt, lane, l32, h, wave;
    int rem;        // keys in the last unit (64 unless N - 1 is ragged)
    i32x8 qf;       // this lane's q8 half row
    int qsc;        // its E8M0 scale
    rsrc_t rk;       // S16: the 16-bit qkv rows of this image (K tiles)
    uint32_t voffk;  // S16: this lane's K-piece offset (row 8 wave + lane / 8, swizzled chunk)
    uint32_t ldb;    // S16: qkv row pitch in bytes
    f32x16 o[2];
    f32x16 negm;
    float m;
    float l4[4];
};

// unit t into ring slot `slot`: one 1-KiB piece per wave (waves 0-3: K rows 16w.., 4-7: V^T
// rows), then 32 B of the scale dwords per wave (lanes 0-7); two vmcnt entries per wave.
// S16: every wave one 1-KiB piece of the 16-bit K tile (rows 8w .. 8w + 7 of the unit, straight
// from qkv: keys 1 + 64t + row, rows past N at 0xFFFFFFF0 = zeros), then waves 0-3 a V^T piece
// and waves 4-7 64 B of the scale dwords (lanes 0-15): two entries per wave as well.
template <bool S16>
__device__ __forceinline__ void f8_issue(F8Ctx<S16>& c, int t, int slot) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (S16) {
        char* base = c.smem + slot * U16SLOT;
        const uint32_t soff = (uint32_t)(1 + 64 * t) * c.ldb;
        const bool ragged = t == c.nt - 1 && c.rem < 64;  // wave-uniform
        if (__builtin_expect(ragged, 0)) {
            const bool ok = c.wave * 8 + (c.lane >> 3) < c.rem;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(c.rk, LDS_PTR(base + c.wave * 1024), 16,
                                                     ok ? c.voffk + soff : 0xFFFFFFF0u, 0, 0, 0);
        } else {
            __builtin_amdgcn_raw_ptr_buffer_load_lds(c.rk, LDS_PTR(base + c.wave * 1024), 16, c.voffk, soff, 0, 0);
        }
        if (c.wave < 4) {
            __builtin_amdgcn_raw_ptr_buffer_load_lds(c.rmine, LDS_PTR(base + 8192 + c.wave * 1024), 16, c.voff,
                                                     (uint32_t)t * c.soff_unit, 0, 0);
        } else if (c.lane < 16) {
            __builtin_amdgcn_raw_ptr_buffer_load_lds(c.rsc, LDS_PTR(base + 12288 + (c.wave - 4) * 64), 4,
                                                     (uint32_t)((c.wave - 4) * 16 + c.lane) * 4, (uint32_t)t * 256, 0,
                                                     0);
        }
        return;
    }
    char* base = c.smem + slot * U8SLOT;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(c.rmine, LDS_PTR(base + c.wave * 1024), 16, c.voff,
                                             (uint32_t)t * c.soff_unit, 0, 0);
    if (c.lane < 8)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(c.rsc, LDS_PTR(base + 8192 + c.wave * 32), 4,
                                                 (uint32_t)(c.wave * 8 + c.lane) * 4, (uint32_t)t * 256, 0, 0);
#endif
}

// 32 bytes of row `row` of a 64-B-row tile image: 16-B chunks h and 2 + h (swizzled), so that
// byte j is element kappa_hw(h, j) of the row (header)
__device__ __forceinline__ i32x8 tile_row(const char* img, int row, int h) {
    const int x = sw8(row);
    const i32x4 a = *(const i32x4*)(img + row * 64 + ((h ^ x) << 4));
    const i32x4 b = *(const i32x4*)(img + row * 64 + (((2 + h) ^ x) << 4));
    return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}

// S^T of the unit in slot image `img` (scales `scw`: the lane's dword of that unit), seeded with init
template <bool S16>
__device__ __forceinline__ void f8_s(f32x16 (&s)[2], const char* img, int scw, const F8Ctx<S16>& c, const f32x16& init) {
    const i32x8 ka = tile_row(img, c.l32, c.h);
    const i32x8 kb = tile_row(img, 32 + c.l32, c.h);
    s[0] = mfma_mx<0>(ka, scw, c.qf, c.qsc, init);
    s[1] = mfma_mx<1>(kb, scw, c.qf, c.qsc, init);
}

// S16: S^T of the unit from its 16-bit K image (32-key blocks kb), q16 the lane's 16-bit q row
template <typename T>
__device__ __forceinline__ void f16_s(f32x16 (&s)[2], const char* img, const typename Mfma<T>::frag (&q16)[4], int l32,
                                      int h, const f32x16& init) {
    typedef typename Mfma<T>::frag frag;
    frag kf[2][4];  // all eight fragment reads first: one LDS round trip, then the MFMA chains
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int j = 0; j < 4; ++j) kf[kb][j] = row_frag<T>(img, kb * 32 + l32, 2 * j + h);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) s[kb] = init;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) s[kb] = Mfma<T>::mma(kf[kb][j], q16[j], s[kb]);
}

__device__ __forceinline__ float f8_rowmax(const f32x16 (&s)[2]) {
    float mx[4] = {s[0][0], s[0][1], s[0][2], s[0][3]};
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = (kb == 0 ? 4 : 0); r < 16; r += 4)
#pragma unroll
            for (int j = 0; j < 4; ++j) mx[j] = fmaxf(mx[j], s[kb][r + j]);
    return xhalf_max(fmaxf(fmaxf(mx[0], mx[1]), fmaxf(mx[2], mx[3])));
}

// keys past the ragged end to -inf: key kb * 32 + acc_row(r, h) of the unit
__device__ __forceinline__ void f8_mask(f32x16 (&s)[2], int rem, int h) {
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r)
            if (kb * 32 + acc_row(r, h) >= rem) s[kb][r] = -INFINITY;
}

// P = exp2(s) of unit scores s (S - m), the lane's partial row sums and the e4m3 P^T operand
__device__ __forceinline__ void f8_exp_pack(const f32x16 (&sc)[2], float (&rsp)[4], i32x8& pf) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        float p[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            p[e] = __builtin_amdgcn_exp2f(sc[0][4 * g + e]);
            p[4 + e] = __builtin_amdgcn_exp2f(sc[1][4 * g + e]);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float pe = p[e] + p[4 + e];
            if (g == 0) rsp[e] = pe;
            else rsp[e] += pe;
        }
        pf[g] = pack4_fp8_unit(p[0], p[1], p[2], p[3]);      // bytes j = 4g .. 4g+3   (t = 0)
        pf[4 + g] = pack4_fp8_unit(p[4], p[5], p[6], p[7]);  // bytes j = 16 + 4g ..   (t = 1)
    }
}

// P(t) from sc (S - m of unit t), O^T += V^T P^T.  As attn_fwd2_kernel, no per-unit row max:
// P = exp2(S - m) is taken against the current reference m and the lane's partial row sum is
// checked instead; only when it exceeds 448 (some P past the e4m3 maximum) is the unit re-done
// with the reference moved to the unit's row max (o, l and the seeded S(t+1) rescaled) before
// P(t) enters O or l.  A reference below the true running max only scales P up: e4m3's relative
// rounding does not depend on the scale, and fewer small P fall into the subnormal range.
template <bool S16>
__device__ __forceinline__ void f8_pv(F8Ctx<S16>& c, f32x16 (&sc)[2], f32x16 (&sn)[2], const char* cur) {
    constexpr int VOFF = S16 ? 8192 : 4096, SOFF = S16 ? 12288 : 8192;  // V^T tile, scales in the slot
    constexpr float LIM = 448.0f;
    float rsp[4];
    i32x8 pf;
    f8_exp_pack(sc, rsp, pf);
    const float tot = (rsp[0] + rsp[1]) + (rsp[2] + rsp[3]);
    if (__any(!(tot <= LIM))) {  // rare: move the reference to the unit's row max and redo P(t)
        const float shift = fmaxf(f8_rowmax(sc), 0.f);
        const float alpha = __builtin_amdgcn_exp2f(-shift);
#pragma unroll
        for (int j = 0; j < 4; ++j) c.l4[j] *= alpha;
#pragma unroll
        for (int db = 0; db < 2; ++db)
#pragma unroll
            for (int r = 0; r < 16; ++r) c.o[db][r] *= alpha;
        c.m += shift;
        const float nm = -c.m;
#pragma unroll
        for (int r = 0; r < 16; ++r) {  // into negm's own registers (tied), as attn_fwd2_kernel
            float x = c.negm[r];
            asm volatile("v_mov_b32 %0, %1" : "+v"(x) : "v"(nm));
            c.negm[r] = x;
        }
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                sc[kb][r] -= shift;
                sn[kb][r] -= shift;
            }
        f8_exp_pack(sc, rsp, pf);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) c.l4[j] += rsp[j];
    const int scw = *(const int*)(cur + SOFF + c.lane * 4);
    const i32x8 va = tile_row(cur + VOFF, c.l32, c.h);
    const i32x8 vb = tile_row(cur + VOFF, 32 + c.l32, c.h);
    c.o[0] = mfma_mx<2>(va, scw, pf, E8M0_ONE, c.o[0]);
    c.o[1] = mfma_mx<3>(vb, scw, pf, E8M0_ONE, c.o[1]);
}

// step t (slot Q = t % 4): S(t+1) into sn beside P(t) / PV(t) from sc.  MASK: the last step of
// a ragged N - 1 (its unit's keys past N to -inf); peeled off the loop so that the steady-state
// step has no branch between the S(t+1) MFMAs and unit t's softmax VALU (a branch there splits
// the scheduling region and serialises the two)
template <typename T, bool S16, int Q, bool MASK = false>
__device__ __forceinline__ void f8_step(F8Ctx<S16>& c, int t, f32x16 (&sc)[2], f32x16 (&sn)[2],
                                        const typename Mfma<T>::frag (&q16)[4]) {
    constexpr int SLOT = S16 ? U16SLOT : U8SLOT;
    wait_vmcnt<2>();               // units t and t+1 landed (own entries; unit t+2 in flight)
    __builtin_amdgcn_s_barrier();  // everyone's; everyone done with step t-1 (slot (t+3) % 4 free)
    f8_issue(c, t + 3 < c.nt ? t + 3 : c.nt - 1, (Q + 3) & 3);
    const char* cur = c.smem + Q * SLOT;
    const char* nxt = c.smem + ((Q + 1) & 3) * SLOT;
    // S(t+1): past the last unit the slot holds a copy of the last unit (the issue clamp), and
    // the result is dropped — the step stays branch-free
    if constexpr (S16)
        f16_s<T>(sn, nxt, q16, c.l32, c.h, c.negm);
    else
        f8_s(sn, nxt, *(const int*)(nxt + 8192 + c.lane * 4), c, c.negm);
    if constexpr (MASK) f8_mask(sc, c.rem, c.h);  // the ragged last unit
    f8_pv(c, sc, sn, cur);
}

// the last step of a ragged sequence, slot (nt - 1) % 4 at run time
template <typename T, bool S16>
__device__ __forceinline__ void f8_step_masked(F8Ctx<S16>& c, int t, f32x16 (&sc)[2], f32x16 (&sn)[2],
                                               const typename Mfma<T>::frag (&q16)[4]) {
    switch (t & 3) {
        case 0: f8_step<T, S16, 0, true>(c, t, sc, sn, q16); break;
        case 1: f8_step<T, S16, 1, true>(c, t, sc, sn, q16); break;
        case 2: f8_step<T, S16, 2, true>(c, t, sc, sn, q16); break;
        default: f8_step<T, S16, 3, true>(c, t, sc, sn, q16); break;
    }
}

// grid B * H * ceil((N - 1) / 256), 512 threads (8 waves x 32 queries 1 + ..)
template <typename T, bool S16>
__global__ __launch_bounds__(512, 1) void attn_fp8mx_kernel(const T* __restrict__ qkv, const uint8_t* __restrict__ q8,
                                                            const uint8_t* __restrict__ qs,
                                                            const uint8_t* __restrict__ k8,
                                                            const uint8_t* __restrict__ vt8,
                                                            const uint32_t* __restrict__ sc, T* __restrict__ out,
                                                            float* __restrict__ lse, int N, int H, int n1p) {
    constexpr int NW = 8, QB = 32 * NW;
    typedef typename Mfma<T>::frag frag;
    __shared__ __attribute__((aligned(16))) char smem[4 * (S16 ? U16SLOT : U8SLOT)];
    F8Ctx<S16> c;
    c.smem = smem;
    c.lane = threadIdx.x & 63;
    c.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    c.h = c.lane >> 5;
    c.l32 = c.lane & 31;
    const int n1 = N - 1;
    const int nq = (n1 + QB - 1) / QB;
    const int tile = xcd_remap(blockIdx.x, gridDim.x);
    const int qblk = tile % nq, bh = tile / nq, b = bh / H, hd = bh % H;
    const int C = H * HD;
    const int64_t ld = 3 * (int64_t)C;
    const int64_t hb = bh;
    c.nt = (n1 + 63) / 64;
    c.rem = n1 - 64 * (c.nt - 1);
    // this lane's query (row qi of the planes = token 1 + qi); rows past N compute on zero rows
    const int qi = qblk * QB + c.wave * 32 + c.l32;
    const bool qok = qi < n1;
    const int qr = qok ? qi : n1 - 1;
    if constexpr (!S16) {
        const uint8_t* qrow = q8 + (hb * n1p + qr) * 64;
        const i32x4 a = *(const i32x4*)(qrow + 16 * c.h), b = *(const i32x4*)(qrow + 32 + 16 * c.h);
        c.qf = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
        c.qsc = qs[(hb * n1p + qr) * 2 + c.h];
    }
    // key 0 (CLS) from the 16-bit qkv, as attn_fwd2_kernel: s0 = q . k0 on the VALU
    const T* Bb = qkv + (int64_t)b * N * ld;
    const T* Qrow = Bb + (int64_t)(1 + qr) * ld + hd * HD;
    frag q16[4], k0[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        q16[s] = *(const frag*)(Qrow + (2 * s + c.h) * 8);
        k0[s] = *(const frag*)(Bb + C + hd * HD + (2 * s + c.h) * 8);
    }
    typedef T t4 __attribute__((ext_vector_type(4)));
    t4 v0[2][4];
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int g = 0; g < 4; ++g) v0[db][g] = *(const t4*)(Bb + 2 * C + hd * HD + db * 32 + 8 * g + 4 * c.h);

    if constexpr (S16) {
        // LDS-DMA sources: every wave a K piece (16-bit rows 8w + lane / 8 of a unit), waves 0-3 a
        // V^T piece (rows 16w + lane / 4), waves 4-7 the scale dwords
        const int prow = (c.wave & 3) * 16 + (c.lane >> 2);
        const uint32_t gchunk = (uint32_t)(((c.lane & 3) ^ sw8(prow)) * 16);
        c.rmine = make_rsrc(vt8 + hb * 64 * n1p, (uint32_t)n1p * 64);
        c.voff = (uint32_t)prow * (uint32_t)n1p + gchunk;
        c.soff_unit = 64u;
        c.ldb = (uint32_t)(ld * sizeof(T));
        c.rk = make_rsrc(Bb, (uint32_t)N * c.ldb);
        const int kr = c.wave * 8 + (c.lane >> 3);
        c.voffk = (uint32_t)kr * c.ldb + (uint32_t)(((c.lane & 7) ^ xsw(kr)) * 16) + (uint32_t)((C + hd * HD) * sizeof(T));
    } else {
        // LDS-DMA sources: waves 0-3 the K plane (rows 16w.. of a unit), 4-7 the V^T plane
        const bool kw = c.wave < 4;
        const int prow = (c.wave & 3) * 16 + (c.lane >> 2);
        const uint32_t gchunk = (uint32_t)(((c.lane & 3) ^ sw8(prow)) * 16);
        c.rmine = kw ? make_rsrc(k8 + hb * n1p * 64, (uint32_t)n1p * 64)
                     : make_rsrc(vt8 + hb * 64 * n1p, (uint32_t)n1p * 64);
        c.voff = kw ? (uint32_t)prow * 64 + gchunk : (uint32_t)prow * (uint32_t)n1p + gchunk;
        c.soff_unit = kw ? 4096u : 64u;
    }
    c.rsc = make_rsrc(sc + hb * (n1p / 64) * 64, (uint32_t)n1p * 4);
    f8_issue(c, 0, 0);
    f8_issue(c, c.nt > 1 ? 1 : 0, 1);
    f8_issue(c, c.nt > 2 ? 2 : c.nt - 1, 2);

    float part = 0.f;
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) part += (float)q16[s][j] * (float)k0[s][j];
    const float s0 = xhalf_sum(part);

    wait_vmcnt<4>();  // unit 0 landed (units 1, 2 in flight)
    __builtin_amdgcn_s_barrier();
    f32x16 sA[2], sB[2];
    if constexpr (S16)
        f16_s<T>(sA, smem, q16, c.l32, c.h, zero16());
    else
        f8_s(sA, smem, *(const int*)(smem + 8192 + c.lane * 4), c, zero16());
    if (c.nt == 1 && c.rem < 64) f8_mask(sA, c.rem, c.h);
    c.m = fmaxf(f8_rowmax(sA), s0);
    c.negm = splat16(-c.m);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) sA[kb][r] -= c.m;
    const float p0 = __builtin_amdgcn_exp2f(s0 - c.m);
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
            for (int e = 0; e < 4; ++e) c.o[db][4 * g + e] = p0 * (float)v0[db][g][e];
    c.l4[0] = c.h == 0 ? p0 : 0.f;
    c.l4[1] = c.l4[2] = c.l4[3] = 0.f;
    if (c.wave >= NW / 2) __builtin_amdgcn_s_setprio(1);  // static priority for the younger half

    // the last step of a ragged N - 1 is peeled (its mask); the loop runs the branch-free steps
    const int nfull = c.rem < 64 ? c.nt - 1 : c.nt;
    int t = 0;
    while (true) {  // unrolled by four: ring slots are immediates
        if (t >= nfull) break;
        f8_step<T, S16, 0>(c, t++, sA, sB, q16);
        if (t >= nfull) break;
        f8_step<T, S16, 1>(c, t++, sB, sA, q16);
        if (t >= nfull) break;
        f8_step<T, S16, 2>(c, t++, sA, sB, q16);
        if (t >= nfull) break;
        f8_step<T, S16, 3>(c, t++, sB, sA, q16);
    }
    if (t < c.nt) {  // ragged: the masked last step, sc in sA when t is even
        if ((t & 1) == 0) f8_step_masked<T, S16>(c, t, sA, sB, q16);
        else f8_step_masked<T, S16>(c, t, sB, sA, q16);
    }
    __builtin_amdgcn_s_setprio(0);
    wait_vmcnt<0>();  // no LDS-DMA may still be landing when the workgroup retires

    const float lt = xhalf_sum((c.l4[0] + c.l4[1]) + (c.l4[2] + c.l4[3]));
    if (qok) {
        const int q = 1 + qi;
        store_row_t21<T>(out + ((int64_t)b * N + q) * C + hd * HD, c.o, 1.0f / lt, c.h);
        if (c.h == 0) lse[(int64_t)bh * N + q] = c.m + __log2f(lt);
    }
}

}  // namespace

extern "C" int64_t dclip_attn_fwd_fp8_workspace(int B, int N, int H) {
    const int64_t n1p = (int64_t)(N - 1 + 63) / 64 * 64;
    // q8, k8, vt8 planes, the q scales, the unit scale dwords, the row-0 pass's partials
    return 3 * (int64_t)B * H * n1p * 64 + (int64_t)B * H * n1p * 2 + (int64_t)B * H * (n1p / 64) * 256 +
           4 * attn_row0_ws_floats(B, N, H) + 256;
}

extern "C" int dclip_attn_fwd_fp8(int dt, const void* qkv, void* o, float* lse, void* ws, int B, int N, int H, int D,
                                  void* stream) {
    DCLIP_HOST_CHECK(D == 64, "dclip_attn_fwd_fp8: head_dim must be 64 (got %d)", D);
    DCLIP_HOST_CHECK(dt == DCLIP_BF16 || dt == DCLIP_F16, "dclip_attn_fwd_fp8: dtype must be f16/bf16");
    DCLIP_HOST_CHECK(B > 0 && N > 0 && H > 0 && H <= 64, "dclip_attn_fwd_fp8: bad problem (B, N > 0, 0 < H <= 64)");
    DCLIP_HOST_CHECK(((uintptr_t)qkv % 16) == 0 && ((uintptr_t)o % 16) == 0 && ((uintptr_t)ws % 256) == 0,
                     "dclip_attn_fwd_fp8: unaligned buffers");
    DCLIP_HOST_CHECK((int64_t)(N + 63) / 64 * 64 * 64 < (1ll << 31), "dclip_attn_fwd_fp8: N too large");
    hipStream_t st = (hipStream_t)stream;
    const int n1p = (N - 1 + 63) / 64 * 64;
    const int64_t plane = (int64_t)B * H * n1p * 64;
    uint8_t* q8 = (uint8_t*)ws;
    uint8_t* k8 = q8 + plane;
    uint8_t* vt8 = k8 + plane;
    uint8_t* qs = vt8 + plane;
    uint32_t* sc = (uint32_t*)(qs + (int64_t)B * H * n1p * 2);  // 4-B aligned: plane, n1p multiples of 64
    float* r0ws = (float*)(sc + (int64_t)B * H * (n1p / 64) * 64);
    // query 0 (the CLS row) by the 16-bit split-key row pass (its partials in the workspace)
    attn_row0_fwd(dt, qkv, o, lse, B, N, H, st, r0ws);
    if (N > 1) {
        const dim3 gp(n1p / 64, H, B);
        const int grid = B * H * ((N - 1 + 255) / 256);
        // DCLIP_OPT_ATTN_FP8_QK 1: S on the fp8 MFMA too (round 3's all-e4m3 kernel)
        const bool s16 = dclip_option(DCLIP_OPT_ATTN_FP8_QK) != 1;
#define FP8_LAUNCH(T, S)                                                                                        \
    fp8mx_pack_kernel<T, !S><<<gp, 256, 0, st>>>((const T*)qkv, q8, qs, k8, vt8, sc, N, H, n1p);                  \
    attn_fp8mx_kernel<T, S><<<grid, 512, 0, st>>>((const T*)qkv, q8, qs, k8, vt8, sc, (T*)o, lse, N, H, n1p);
        if (dt == DCLIP_BF16) {
            if (s16) { FP8_LAUNCH(bf16, true) } else { FP8_LAUNCH(bf16, false) }
        } else {
            if (s16) { FP8_LAUNCH(f16, true) } else { FP8_LAUNCH(f16, false) }
        }
#undef FP8_LAUNCH
    }
    DCLIP_LAUNCH_CHECK();
    return 0;
}
