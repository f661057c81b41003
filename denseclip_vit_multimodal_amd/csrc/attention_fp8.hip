// fp8 (OCP e4m3) attention forward for inference — BASELINE config 5 ("fp8 MFMA attention").
//
// Same contract as dclip_attn_fwd (reference: the nn.MultiheadAttention core of
// ResidualAttentionBlock.attention, models.py:287-289; q columns of the packed qkv pre-multiplied
// by d^-0.5 * log2(e)), computed on the block-scaled gfx950 MFMA
// v_mfma_scale_f32_32x32x64_f8f6f4 with unit (E8M0 = 127) block scales, which runs at twice the
// bf16 rate: one instruction covers K = 64, i.e. a whole head dimension or 64 keys.
//
// Three launches:
//   1. fp8_amax_kernel   per-(image, q/k/v, head) amax of the 16-bit qkv (integer atomicMax on
//                        the float bits: all values are >= 0)
//   2. fp8_pack_kernel   quantise with scale 448 / amax (saturating) into a per-head layout:
//                          q8, k8 [b][h][Npad][64] bytes      (token rows, 64 B each)
//                          vt8   [b][h][64][Npad] bytes       (V transposed, keys permuted per
//                                                              64-key unit, see kappa() below)
//                        rows / keys past N are zero
//   3. attn_fp8_kernel   flash forward: 8 waves x 32 queries per workgroup; per 64-key unit the
//                        K tile (4 KB) and V^T tile (4 KB) are staged in LDS (double-buffered,
//                        prefetched into registers one unit ahead); per wave
//                          S^T = K Q^T          2 MFMAs (keys 0-31, 32-63), lane = query
//                          online softmax       log2 domain, one cross-half max per unit
//                          O^T += V^T P^T       2 MFMAs (d 0-31, 32-63); P^T straight from the
//                                               S^T accumulators, converted to fp8 in registers
//
// Operand maps.  For the 32x32x64 f8f6f4 MFMA a lane (r = lane & 31, half = lane >> 5) holds
// 32 bytes of row r of A (column r of B); byte j of half `half` is one K index kappa(half, j),
// the SAME for A and B.  Only that sameness is relied on: every contraction below assigns its
// logical K index to (half, j) identically on both sides.  For S^T = K Q^T the K index is the
// head dim d = 32 half + j (both operands are plain 64-byte token rows).  For O^T = V^T P^T it
// is the key: the S^T accumulator of key sub-tile t has key (reg & 3) + 8 (reg >> 2) + 4 half
// in register reg (the dtype-independent C/D map), so the lane's 32 P values are used as
// bytes j = 16 t + reg, which makes slot (half, j) = key kappa(half, j) below; fp8_pack_kernel
// writes V^T with that permutation inside every 64-key unit so the V^T operand is 32
// contiguous bytes too.
#include "common.h"

#include <type_traits>

namespace {

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

constexpr float FP8_MAX = 448.0f;
constexpr int FP8_FMT_E4M3 = 0;  // f8f6f4 format code of OCP e4m3
constexpr int E8M0_ONE = 127;    // block scale 2^0

__device__ __forceinline__ int kappa(int half, int j) {  // key within a 64-key unit
    const int t = j >> 4, reg = j & 15;
    return 32 * t + (reg & 3) + 8 * (reg >> 2) + 4 * half;
}

__device__ __forceinline__ f32x16 mfma_fp8(i32x8 a, i32x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, FP8_FMT_E4M3, FP8_FMT_E4M3, 0, E8M0_ONE, 0,
                                                           E8M0_ONE);
}

// 4 floats -> 4 e4m3 bytes of one dword (saturated to +-448 first: the convert does not clamp)
__device__ __forceinline__ int pack4_fp8(float a, float b, float c, float d) {
    a = fminf(fmaxf(a, -FP8_MAX), FP8_MAX);
    b = fminf(fmaxf(b, -FP8_MAX), FP8_MAX);
    c = fminf(fmaxf(c, -FP8_MAX), FP8_MAX);
    d = fminf(fmaxf(d, -FP8_MAX), FP8_MAX);
    int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
    return __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
}
// the same for values known to lie in [0, 1] (softmax probabilities): no clamp needed
__device__ __forceinline__ int pack4_fp8_unit(float a, float b, float c, float d) {
    int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
    return __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
}

// ---------------------------------------------------------------------------- 1. amax
// grid (ceil(N / 64), B), 256 threads; amax[b][which][h] (float bits as int, pre-zeroed)
template <typename T>
__global__ void __launch_bounds__(256) fp8_amax_kernel(const T* __restrict__ qkv, int* __restrict__ amax, int N,
                                                       int H) {
    __shared__ int red[3 * 64];
    const int C = H * 64, ncol8 = 3 * C / 8;
    const int b = blockIdx.y, t0 = blockIdx.x * 64;
    for (int i = threadIdx.x; i < 3 * H; i += 256) red[i] = 0;
    __syncthreads();
    const int ntok = min(64, N - t0);
    // a thread keeps one 8-column chunk (fixed head) while it walks tokens when 256 % ncol8 == 0;
    // in general it re-derives the chunk per item
    for (int c8 = threadIdx.x; c8 < ncol8; c8 += 256) {
        float m = 0.f;
        const T* p = qkv + ((int64_t)b * N + t0) * 3 * C + c8 * 8;
        for (int t = 0; t < ntok; ++t) {
            const uint4 raw = *(const uint4*)(p + (int64_t)t * 3 * C);
            const T* e = (const T*)&raw;
#pragma unroll
            for (int k = 0; k < 8; ++k) m = fmaxf(m, fabsf((float)e[k]));
        }
        const int col = c8 * 8, which = col / C, h = (col % C) / 64;
        atomicMax(&red[which * H + h], __float_as_int(m));
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 3 * H; i += 256) atomicMax(&amax[b * 3 * H + i], red[i]);
}

// the same with one thread per (8-column chunk, token parity): blockDim = 2 * ncol8 (<= 1024),
// every thread walks 32 of the 64 tokens with 8 loads in flight (the loop above keeps one
// load in flight per thread and leaves 256 - ncol8 % 256 threads idle on its last pass)
template <typename T>
__global__ void __launch_bounds__(1024) fp8_amax2_kernel(const T* __restrict__ qkv, int* __restrict__ amax, int N,
                                                         int H) {
    __shared__ int red[3 * 64];
    const int C = H * 64, ncol8 = 3 * C / 8;
    const int b = blockIdx.y, t0 = blockIdx.x * 64;
    const int c8 = threadIdx.x % ncol8, par = threadIdx.x / ncol8;
    for (int i = threadIdx.x; i < 3 * H; i += blockDim.x) red[i] = 0;
    __syncthreads();
    const int ntok = min(64, N - t0);
    const T* p = qkv + ((int64_t)b * N + t0) * 3 * C + c8 * 8;
    float m = 0.f;
#pragma unroll 8
    for (int t = par; t < ntok; t += 2) {
        const uint4 raw = *(const uint4*)(p + (int64_t)t * 3 * C);
        const T* e = (const T*)&raw;
#pragma unroll
        for (int k = 0; k < 8; ++k) m = fmaxf(m, fabsf((float)e[k]));
    }
    const int col = c8 * 8, which = col / C, h = (col % C) / 64;
    atomicMax(&red[which * H + h], __float_as_int(m));
    __syncthreads();
    for (int i = threadIdx.x; i < 3 * H; i += blockDim.x) atomicMax(&amax[b * 3 * H + i], red[i]);
}

// ---------------------------------------------------------------------------- 2. pack
// grid (Npad / 64, H, B), 256 threads: one 64-token unit of one head
template <typename T>
__global__ void __launch_bounds__(256) fp8_pack_kernel(const T* __restrict__ qkv, const int* __restrict__ amax,
                                                       uint8_t* __restrict__ q8, uint8_t* __restrict__ k8,
                                                       uint8_t* __restrict__ vt8, int N, int H, int Npad) {
    __shared__ float vs[64][65];
    const int C = H * 64;
    const int unit = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
    const int t0 = unit * 64;
    const int tid = threadIdx.x;
    const float* am = (const float*)amax + b * 3 * H;
    const float aq = am[h], ak = am[H + h], av = am[2 * H + h];
    const float sq = aq > 0.f ? FP8_MAX / aq : 1.f;
    const float sk = ak > 0.f ? FP8_MAX / ak : 1.f;
    const float sv = av > 0.f ? FP8_MAX / av : 1.f;
    const int64_t hb = (int64_t)b * H + h;
    // q and k rows: thread -> (token, 16-wide d chunk)
    {
        const int t = tid >> 2, d0 = (tid & 3) * 16;
        const int tok = t0 + t;
        i32x4 oq = {0, 0, 0, 0}, ok = {0, 0, 0, 0};
        float v[16];
        if (tok < N) {
            const T* row = qkv + ((int64_t)b * N + tok) * 3 * C + h * 64 + d0;
            const uint4 r0 = *(const uint4*)row, r1 = *(const uint4*)(row + 8);
            const T* e0 = (const T*)&r0;
            const T* e1 = (const T*)&r1;
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = (float)e0[k] * sq, v[8 + k] = (float)e1[k] * sq;
#pragma unroll
            for (int k = 0; k < 4; ++k) oq[k] = pack4_fp8(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
            const uint4 s0 = *(const uint4*)(row + C), s1 = *(const uint4*)(row + C + 8);
            const T* f0 = (const T*)&s0;
            const T* f1 = (const T*)&s1;
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = (float)f0[k] * sk, v[8 + k] = (float)f1[k] * sk;
#pragma unroll
            for (int k = 0; k < 4; ++k) ok[k] = pack4_fp8(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
            const uint4 u0 = *(const uint4*)(row + 2 * C), u1 = *(const uint4*)(row + 2 * C + 8);
            const T* g0 = (const T*)&u0;
            const T* g1 = (const T*)&u1;
#pragma unroll
            for (int k = 0; k < 8; ++k) vs[t][d0 + k] = (float)g0[k] * sv, vs[t][d0 + 8 + k] = (float)g1[k] * sv;
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k) vs[t][d0 + k] = 0.f;
        }
        *(i32x4*)(q8 + (hb * Npad + tok) * 64 + d0) = oq;
        *(i32x4*)(k8 + (hb * Npad + tok) * 64 + d0) = ok;
    }
    __syncthreads();
    // V^T: thread -> (d, 16 consecutive permuted key slots)
    {
        const int d = tid >> 2, s0 = (tid & 3) * 16;
        i32x4 o;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float e[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int s = s0 + 4 * k + q;  // slot = 32 half + j
                e[q] = vs[kappa(s >> 5, s & 31)][d];
            }
            o[k] = pack4_fp8(e[0], e[1], e[2], e[3]);
        }
        *(i32x4*)(vt8 + (hb * 64 + d) * Npad + t0 + s0) = o;
    }
}

// ---------------------------------------------------------------------------- 3. attention
// grid (ceil(N / (32 NW)), H, B), 64 NW threads (NW waves x 32 queries)
template <typename T, int NW>
__global__ void __launch_bounds__(64 * NW) attn_fp8_kernel(const uint8_t* __restrict__ q8, const uint8_t* __restrict__ k8,
                                                       const uint8_t* __restrict__ vt8, const int* __restrict__ amax,
                                                       T* __restrict__ o, float* __restrict__ lse, int N, int H,
                                                       int Npad, int q0) {
    __shared__ __attribute__((aligned(16))) uint8_t sm[2][2][64 * 64];  // [buf][K | V^T][64 rows x 64 B]
    const int h = blockIdx.y, b = blockIdx.z;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int r = lane & 31, half = lane >> 5;
    const int q = q0 + blockIdx.x * (32 * NW) + wave * 32 + r;  // this lane's query (column of S^T)
    const int64_t hb = (int64_t)b * H + h;
    const float* am = (const float*)amax + b * 3 * H;
    const float dq = am[h] > 0.f ? am[h] / FP8_MAX : 1.f;
    const float dk = am[H + h] > 0.f ? am[H + h] / FP8_MAX : 1.f;
    const float dv = am[2 * H + h] > 0.f ? am[2 * H + h] / FP8_MAX : 1.f;
    const float sscale = dq * dk;  // S (log2 domain) = sscale * (q8 . k8)

    // Q^T operand: 32 bytes of this lane's query row (zero rows past N were packed as zeros)
    const uint8_t* qrow = q8 + (hb * Npad + min(q, Npad - 1)) * 64 + 32 * half;
    const i32x8 qf = *(const i32x8*)qrow;

    // cooperative tile loads of a unit's K tile (4 KB contiguous) and V^T tile (64 rows x 64 B):
    // NW = 8: threads 0-255 K, 256-511 V^T, 16 B each; NW = 4: every thread 16 B of both
    static_assert(NW == 4 || NW == 8, "4 or 8 waves");
    const int t256 = tid & 255;
    const uint8_t* ksrc = k8 + hb * Npad * 64 + t256 * 16;
    const int vd = t256 >> 2, vpart = (tid & 3) * 16;
    const uint8_t* vsrc = vt8 + (hb * 64 + vd) * Npad + vpart;
    const int nunit = Npad / 64;
    struct Pre { i32x4 k, v; };
    auto load_unit = [&](int u) -> Pre {
        Pre p;
        if (NW == 4 || tid < 256) p.k = *(const i32x4*)(ksrc + (int64_t)u * 4096);
        if (NW == 4 || tid >= 256) p.v = *(const i32x4*)(vsrc + u * 64);
        return p;
    };
    auto store_unit = [&](int buf, const Pre& p) {
        if (NW == 4 || tid < 256) *(i32x4*)(&sm[buf][0][t256 * 16]) = p.k;
        if (NW == 4 || tid >= 256) *(i32x4*)(&sm[buf][1][vd * 64 + vpart]) = p.v;
    };

    f32x16 o0, o1;
#pragma unroll
    for (int i = 0; i < 16; ++i) o0[i] = 0.f, o1[i] = 0.f;
    float m = -INFINITY, l = 0.f;

    Pre pre = load_unit(0);
    store_unit(0, pre);
    if (nunit > 1) pre = load_unit(1);
    __syncthreads();
    // one 64-key unit; TAIL: the last unit when N is not a multiple of 64 (keys >= N masked).
    // VALU per unit and lane is the limit at the fp8 MFMA rate (4 MFMAs = 256 cycles against
    // 32 exponentials = 256 issue cycles), so: raw v_exp_f32 (no denormal range-reduction
    // sequence), the dequantisation scale folded into the exponent's FMA, the maximum taken
    // on the raw scores (sscale > 0: max(raw) * sscale == max(raw * sscale) exactly), the mask
    // only in the peeled tail unit, and the O / l rescale skipped when no lane's maximum moved
    // (alpha == 1 exactly then: the skipped multiplications were identities).
    auto unit = [&](int u, auto tail_tag) {
        constexpr bool TAIL = decltype(tail_tag)::value;
        const int buf = u & 1;
        if (u + 1 < nunit) {
            store_unit(buf ^ 1, pre);  // buffer buf^1 was last read in unit u-1 (barrier below)
            if (u + 2 < nunit) pre = load_unit(u + 2);
        }
        const uint8_t* ks = sm[buf][0];
        const uint8_t* vs = sm[buf][1];
        // S^T tiles: A = K rows (keys 0-31 / 32-63 of the unit), B = Q^T
        const i32x8 ka = *(const i32x8*)(ks + r * 64 + 32 * half);
        const i32x8 kb = *(const i32x8*)(ks + (32 + r) * 64 + 32 * half);
        f32x16 zero;
#pragma unroll
        for (int i = 0; i < 16; ++i) zero[i] = 0.f;
        f32x16 s0 = mfma_fp8(ka, qf, zero);
        f32x16 s1 = mfma_fp8(kb, qf, zero);
        if constexpr (TAIL) {
            const int kbase = u * 64 + 4 * half;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int kr = (i & 3) + 8 * (i >> 2);
                if (kbase + kr >= N) s0[i] = -INFINITY;
                if (kbase + 32 + kr >= N) s1[i] = -INFINITY;
            }
        }
        float mx = -INFINITY;
#pragma unroll
        for (int i = 0; i < 16; ++i) mx = fmaxf(mx, fmaxf(s0[i], s1[i]));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));  // the other half holds the query's other keys
        const float mnew = fmaxf(m, mx * sscale);
        if (__builtin_amdgcn_read_exec() & __ballot(mnew > m)) {  // some lane's maximum moved
            const float alpha = __builtin_amdgcn_exp2f(m - mnew);
            l *= alpha;
#pragma unroll
            for (int i = 0; i < 16; ++i) o0[i] *= alpha, o1[i] *= alpha;
            m = mnew;
        }
        const float nm = -mnew;
        float rs = 0.f;
        i32x8 pf;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const float p0 = __builtin_amdgcn_exp2f(fmaf(s0[4 * g], sscale, nm));
            const float p1 = __builtin_amdgcn_exp2f(fmaf(s0[4 * g + 1], sscale, nm));
            const float p2 = __builtin_amdgcn_exp2f(fmaf(s0[4 * g + 2], sscale, nm));
            const float p3 = __builtin_amdgcn_exp2f(fmaf(s0[4 * g + 3], sscale, nm));
            const float p4 = __builtin_amdgcn_exp2f(fmaf(s1[4 * g], sscale, nm));
            const float p5 = __builtin_amdgcn_exp2f(fmaf(s1[4 * g + 1], sscale, nm));
            const float p6 = __builtin_amdgcn_exp2f(fmaf(s1[4 * g + 2], sscale, nm));
            const float p7 = __builtin_amdgcn_exp2f(fmaf(s1[4 * g + 3], sscale, nm));
            rs += (p0 + p1) + (p2 + p3) + (p4 + p5) + (p6 + p7);
            pf[g] = pack4_fp8_unit(p0, p1, p2, p3);      // bytes j = 4g .. 4g+3   (t = 0)
            pf[4 + g] = pack4_fp8_unit(p4, p5, p6, p7);  // bytes j = 16 + 4g ..   (t = 1)
        }
        l += rs;
        // O^T += V^T P^T: A = V^T rows d (0-31 / 32-63), permuted key slots
        const i32x8 va = *(const i32x8*)(vs + r * 64 + 32 * half);
        const i32x8 vb = *(const i32x8*)(vs + (32 + r) * 64 + 32 * half);
        o0 = mfma_fp8(va, pf, o0);
        o1 = mfma_fp8(vb, pf, o1);
        __syncthreads();  // everyone is done with sm[buf] and the next unit's tile is stored
    };
    const int nfull = N / 64;  // units with 64 valid keys; a ragged last unit is peeled
    for (int u = 0; u < nfull; ++u) unit(u, std::false_type{});
    if (nfull < nunit) unit(nfull, std::true_type{});
    l += __shfl_xor(l, 32, 64);
    if (q >= N) return;
    const float inv = dv / l;
    T* orow = o + ((int64_t)b * N + q) * (H * 64) + h * 64;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const int d = 8 * g + 4 * half;
        T v0[4], v1[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v0[e] = (T)(o0[4 * g + e] * inv), v1[e] = (T)(o1[4 * g + e] * inv);
        *(uint2*)(orow + d) = *(const uint2*)v0;
        *(uint2*)(orow + 32 + d) = *(const uint2*)v1;
    }
    if (half == 0) lse[hb * N + q] = m + log2f(l);
}

}  // namespace

extern "C" int64_t dclip_attn_fwd_fp8_workspace(int B, int N, int H) {
    const int64_t npad = (N + 63) / 64 * 64;
    return 3 * (int64_t)B * H * npad * 64 + (int64_t)B * 3 * H * 4;  // q8, k8, vt8, amax
}

extern "C" int dclip_attn_fwd_fp8(int dt, const void* qkv, void* o, float* lse, void* ws, int B, int N, int H, int D,
                                  void* stream) {
    DCLIP_HOST_CHECK(D == 64, "dclip_attn_fwd_fp8: head_dim must be 64 (got %d)", D);
    DCLIP_HOST_CHECK(dt == DCLIP_BF16 || dt == DCLIP_F16, "dclip_attn_fwd_fp8: dtype must be f16/bf16");
    DCLIP_HOST_CHECK(B > 0 && N > 0 && H > 0 && H <= 64, "dclip_attn_fwd_fp8: bad problem (B, N > 0, 0 < H <= 64)");
    DCLIP_HOST_CHECK(((uintptr_t)qkv % 16) == 0 && ((uintptr_t)o % 8) == 0 && ((uintptr_t)ws % 256) == 0,
                     "dclip_attn_fwd_fp8: unaligned buffers");
    const int npad = (N + 63) / 64 * 64;
    const int64_t plane = (int64_t)B * H * npad * 64;
    uint8_t* q8 = (uint8_t*)ws;
    uint8_t* k8 = q8 + plane;
    uint8_t* vt8 = k8 + plane;
    int* amax = (int*)(vt8 + plane);  // plane is a multiple of 4096 bytes
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(amax, 0, (size_t)B * 3 * H * 4, st) != hipSuccess) {
        dclip_set_error("dclip_attn_fwd_fp8: memset failed");
        return DCLIP_ERR_HIP;
    }
    // CLS split (N = 1 + 256k, the benchmark's 8193): query 0 by the bf16 row pass of the
    // 16-bit forward, queries 1..N-1 as full 256-query blocks — no near-empty last block
    // (at N = 8193 that block held 1 query and cost a full key sweep: 33 blocks -> 32, and
    // B*H*32 workgroups fill whole rounds of 2 workgroups per CU)
    const bool cls = N >= 257 && (N - 1) % 256 == 0;
    const int q0 = cls ? 1 : 0;
    // 4-wave workgroups (128 queries; DCLIP_OPT_ATTN_FWD_WAVES 4) or 8-wave (256 queries)
    const int fnw = dclip_option(DCLIP_OPT_ATTN_FWD_WAVES) == 4 ? 4 : 8;
    const dim3 ga((N + 63) / 64, B), gp(npad / 64, H, B), gf((N - q0 + 32 * fnw - 1) / (32 * fnw), H, B);
    if (cls) attn_row0_fwd(dt, qkv, o, lse, B, N, H, st);
    const int ncol8 = 3 * H * 64 / 8;
    const bool amax2 = 2 * ncol8 <= 1024 && (2 * ncol8) % 64 == 0;
    if (dt == DCLIP_BF16) {
        if (amax2) fp8_amax2_kernel<bf16><<<ga, 2 * ncol8, 0, st>>>((const bf16*)qkv, amax, N, H);
        else fp8_amax_kernel<bf16><<<ga, 256, 0, st>>>((const bf16*)qkv, amax, N, H);
        fp8_pack_kernel<bf16><<<gp, 256, 0, st>>>((const bf16*)qkv, amax, q8, k8, vt8, N, H, npad);
        if (fnw == 4) attn_fp8_kernel<bf16, 4><<<gf, 256, 0, st>>>(q8, k8, vt8, amax, (bf16*)o, lse, N, H, npad, q0);
        else attn_fp8_kernel<bf16, 8><<<gf, 512, 0, st>>>(q8, k8, vt8, amax, (bf16*)o, lse, N, H, npad, q0);
    } else {
        if (amax2) fp8_amax2_kernel<f16><<<ga, 2 * ncol8, 0, st>>>((const f16*)qkv, amax, N, H);
        else fp8_amax_kernel<f16><<<ga, 256, 0, st>>>((const f16*)qkv, amax, N, H);
        fp8_pack_kernel<f16><<<gp, 256, 0, st>>>((const f16*)qkv, amax, q8, k8, vt8, N, H, npad);
        if (fnw == 4) attn_fp8_kernel<f16, 4><<<gf, 256, 0, st>>>(q8, k8, vt8, amax, (f16*)o, lse, N, H, npad, q0);
        else attn_fp8_kernel<f16, 8><<<gf, 512, 0, st>>>(q8, k8, vt8, amax, (f16*)o, lse, N, H, npad, q0);
    }
    DCLIP_LAUNCH_CHECK();
    return 0;
}
