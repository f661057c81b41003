// Shared device helpers for the DenseCLIP gfx950 kernels.
//
// Data types on this path: activations/weights feeding MFMA are bf16 or fp16
// (fp32 accumulate); the residual stream, LayerNorm statistics and all gradient
// sums are fp32.  Wave = 64 lanes; MFMA shape v_mfma_f32_32x32x16_{bf16,f16}.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dclip.h"

typedef __bf16 bf16;
typedef _Float16 f16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short i16x4 __attribute__((ext_vector_type(4)));

#define LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))

#define DCLIP_HOST_CHECK(cond, ...)                                   \
    do {                                                              \
        if (!(cond)) {                                                \
            dclip_set_error(__VA_ARGS__);                             \
            return DCLIP_ERR_ARG;                                     \
        }                                                             \
    } while (0)

#define DCLIP_LAUNCH_CHECK()                                          \
    do {                                                              \
        hipError_t e_ = hipGetLastError();                            \
        if (e_ != hipSuccess) {                                       \
            dclip_set_error("HIP launch failed: %s", hipGetErrorString(e_)); \
            return DCLIP_ERR_HIP;                                     \
        }                                                             \
    } while (0)

void dclip_set_error(const char* fmt, ...);
int dclip_option(int id);  // current value of a dclip_set_option knob (0 = default)

// ----------------------------------------------------------------------------- scalar io
template <typename T> __device__ __forceinline__ float to_f32(T v) { return (float)v; }
template <typename T> __device__ __forceinline__ T from_f32(float v) { return (T)v; }

// load/store of one element of a runtime-typed buffer (host dispatches on dtype
// where it matters for speed; this is for the cold paths)
__device__ __forceinline__ float load_dyn(const void* p, int dt, int64_t i) {
    if (dt == DCLIP_F32) return ((const float*)p)[i];
    if (dt == DCLIP_F16) return (float)((const f16*)p)[i];
    return (float)((const bf16*)p)[i];
}
__device__ __forceinline__ void store_dyn(void* p, int dt, int64_t i, float v) {
    if (dt == DCLIP_F32) ((float*)p)[i] = v;
    else if (dt == DCLIP_F16) ((f16*)p)[i] = (f16)v;
    else ((bf16*)p)[i] = (bf16)v;
}

// ----------------------------------------------------------------------------- wave ops
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// c + the sum of an 8-element fragment (four v_dot2c_f32 against packed ones)
__device__ __forceinline__ float frag_sum8(bf16x8 v, float c) {
    typedef bf16 b2 __attribute__((ext_vector_type(2)));
    const b2 one = {(bf16)1.f, (bf16)1.f};
#pragma unroll
    for (int p = 0; p < 4; ++p) c = __builtin_amdgcn_fdot2_f32_bf16(b2{v[2 * p], v[2 * p + 1]}, one, c, false);
    return c;
}
__device__ __forceinline__ float frag_sum8(f16x8 v, float c) {
    typedef f16 h2 __attribute__((ext_vector_type(2)));
    const h2 one = {(f16)1.f, (f16)1.f};
#pragma unroll
    for (int p = 0; p < 4; ++p) c = __builtin_amdgcn_fdot2(h2{v[2 * p], v[2 * p + 1]}, one, c, false);
    return c;
}

// ----------------------------------------------------------------------------- MFMA
template <typename T> struct Mfma;
template <> struct Mfma<bf16> {
    typedef bf16x8 frag;
    static __device__ __forceinline__ f32x16 mma(frag a, frag b, f32x16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    }
};
template <> struct Mfma<f16> {
    typedef f16x8 frag;
    static __device__ __forceinline__ f32x16 mma(frag a, frag b, f32x16 c) {
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
    }
};

// v_mfma_f32_16x16x32_{bf16,f16}: lane l holds A[l & 15][8(l >> 4) + j], B[8(l >> 4) + j][l & 15]
// and D[4(l >> 4) + e][l & 15]
template <typename T> struct Mfma16;
template <> struct Mfma16<bf16> {
    static __device__ __forceinline__ f32x4 mma(bf16x8 a, bf16x8 b, f32x4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    }
};
template <> struct Mfma16<f16> {
    static __device__ __forceinline__ f32x4 mma(f16x8 a, f16x8 b, f32x4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
    }
};

// s_waitcnt vmcnt(N) only (expcnt / lgkmcnt left at their maxima), N a compile-time constant
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt(0x0F70 | (N & 15) | ((N >> 4) << 14));
}

// QuickGELU z * sigmoid(1.702 z) and its derivative, on v_exp_f32 + v_rcp_f32 (each ~1 ulp) — an
// IEEE f32 division here costs ~12 VALU instructions per element and dominated the GELU GEMM
// epilogues.  Saturates correctly: exp2 -> inf gives rcp 0, exp2 -> 0 gives rcp 1.
__device__ __forceinline__ float quick_gelu_sigmoid(float z) {
    return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-1.702f * 1.4426950408889634f * z));
}
__device__ __forceinline__ float quick_gelu(float z) {
    return z * quick_gelu_sigmoid(z);
}
__device__ __forceinline__ float quick_gelu_grad(float z) {
    const float s = quick_gelu_sigmoid(z);
    return s + 1.702f * z * s * (1.0f - s);
}

// buffer resource over [p, p + bytes): buffer loads past the end read 0 (LDS-DMA staging)
typedef __amdgpu_buffer_rsrc_t rsrc_t;

__device__ __forceinline__ rsrc_t make_rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

// GEMM output scale: v, times *p when p is set (a device-resident factor such as the 1/s of a
// dclip_grad_scale pair, read once per workgroup — no host round trip for fp16 gradients)
struct Alpha {
    float v;
    const float* p;
    __host__ __device__ Alpha(float v_ = 1.f, const float* p_ = nullptr) : v(v_), p(p_) {}
    __device__ __forceinline__ float get() const { return p ? v * *p : v; }
};

// Power-of-two fp16 gradient scale from a grid-wide |x| maximum, on the device.  st = {s, 1/s,
// amax bits, arrivals}; st[2], st[3] are zero on entry.  Every workgroup (NW waves) joins its
// maximum m (|x| as uint32 bits: they order like the floats, NaN / inf above every finite value);
// the last workgroup to arrive writes st[0] = s = 2^clamp(floor(log2(target / amax)), -60, 60),
// st[1] = 1/s (s = 1 for an all-zero or non-finite maximum) and clears st[2], st[3] for the next
// use.  (dclip_grad_scale, dclip_add_readout_amax.)
template <int NW>
__device__ __forceinline__ void scale_finish(uint32_t m, float target, float* __restrict__ st) {
    for (int o = 32; o >= 1; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
    __shared__ uint32_t red[NW];
    __shared__ bool last;
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        m = red[0];
#pragma unroll
        for (int w = 1; w < NW; ++w) m = max(m, red[w]);
        uint32_t* stu = (uint32_t*)st;
        atomicMax(stu + 2, m);
        __threadfence();
        last = atomicAdd(stu + 3, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (last && threadIdx.x == 0) {
        __threadfence();
        uint32_t* stu = (uint32_t*)st;
        const uint32_t bits = atomicMax(stu + 2, 0u);
        int e = 0;
        if (bits != 0 && bits < 0x7f800000u) {
            const double l = floor(log2((double)target / (double)__uint_as_float(bits)));
            e = (int)fmin(60.0, fmax(-60.0, l));
        }
        st[0] = ldexpf(1.f, e);
        st[1] = ldexpf(1.f, -e);
        atomicExch(stu + 2, 0u);
        atomicExch(stu + 3, 0u);
    }
}

// Delayed power-of-two fp16 gradient scale of one gradient site (dclip.h, the *_scaled casts),
// without fences or an arrival counter: st = [3][DS_SHARDS] |x|-maximum shards (uint32 bits of
// positive floats) + [3] used scales.  Use k casts with the scale of use k-1's maximum (shards
// (k+2) % 3), joins its own maximum into shards k % 3 (one no-return atomic per workgroup, spread
// over the shards) and clears shards (k+1) % 3 for use k+1 (nobody reads them during use k).
// A previous maximum that is 0 or not finite (an inf from an overflow upstream) keeps the scale
// that use k-1 itself used.
constexpr int DS_SHARDS = 64;
constexpr int DS_STATE_FLOATS = 3 * DS_SHARDS + 4;
static_assert(DS_STATE_FLOATS == DCLIP_DS_STATE_FLOATS, "dclip.h state size");

// the scale of use k, computed by every calling wave (one load per lane, L2-resident)
__device__ __forceinline__ float ds_scale_of_use(const float* __restrict__ st, int use, float target) {
    const uint32_t* sh = (const uint32_t*)st + ((use + 2) % 3) * DS_SHARDS;
    uint32_t m = sh[threadIdx.x & 63];
    for (int o = 32; o >= 1; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
    if (m == 0 || m >= 0x7f800000u) return st[3 * DS_SHARDS + (use + 2) % 3];
    const double l = floor(log2((double)target / (double)__uint_as_float(m)));
    return ldexpf(1.f, (int)fmin(60.0, fmax(-60.0, l)));
}

// workgroup 0: publish (s, 1/s) for the consumers, record s as use k's scale, clear shards k+1
__device__ __forceinline__ void ds_begin(float* __restrict__ st, int use, float s, float* __restrict__ spair) {
    if (blockIdx.x != 0 || threadIdx.x >= 64) return;
    ((uint32_t*)st)[((use + 1) % 3) * DS_SHARDS + threadIdx.x] = 0u;
    if (threadIdx.x == 0) {
        spair[0] = s;
        spair[1] = 1.f / s;
        st[3 * DS_SHARDS + use % 3] = s;
    }
}

// the workgroup's (NW waves) |x| maximum m joined into use k's shards
template <int NW>
__device__ __forceinline__ void ds_end(uint32_t m, float* __restrict__ st, int use) {
    for (int o = 32; o >= 1; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
    __shared__ uint32_t red[NW];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        m = red[0];
#pragma unroll
        for (int w = 1; w < NW; ++w) m = max(m, red[w]);
        if (m != 0) atomicMax((uint32_t*)st + (use % 3) * DS_SHARDS + blockIdx.x % DS_SHARDS, m);
    }
}

// bijective XCD-aware remap of a linear block id (8 XCDs, round-robin dispatch):
// consecutive logical tiles land on the same XCD so they share its L2.
__device__ __forceinline__ int xcd_remap(int bid, int nblk) {
    const int q = nblk / 8, r = nblk % 8;
    const int xcd = bid % 8, loc = bid / 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

// query 0 (CLS row) of the 16-bit forward: split-key row pass + merge (attention.hip); the
// partials go to pws (attn_row0_ws_floats floats) or, when null, into rows 1.. of o (N >= 257)
void attn_row0_fwd(int dt, const void* qkv, void* o, float* lse, int B, int N, int H, hipStream_t st,
                   float* pws = nullptr);
inline int64_t attn_row0_ws_floats(int B, int N, int H) { return (int64_t)B * H * ((N + 1023) / 1024) * 4 * 66; }
// CLS-split dK/dV pass with 64 keys per wave and AGPR accumulators (attention_dkdv6.hip); r0q
// receives one dQ_0 partial (64 floats) per key block
void attn_bwd_dkdv6_launch(int dt, const void* qkv, const void* dout, const float* lse, const float* delta,
                           const float* nlse, const float* ndelta, void* dqkv, int B, int N, int H, float dk_scale,
                           float* r0q, hipStream_t st);
// the software-pipelined dkdv6 (DCLIP_OPT_ATTN_BWD_BLOCK 7), bitwise equal to it
void attn_bwd_dkdv7_launch(int dt, const void* qkv, const void* dout, const float* lse, const float* delta,
                           const float* nlse, const float* ndelta, void* dqkv, int B, int N, int H, float dk_scale,
                           float* r0q, hipStream_t st);
// its fp8 form (configs[4]: dV, dK on the block-scaled e4m3 MFMA; attention_dkdv6.hip): the pack of
// the slices' Q^T / dO^T e4m3 images into f8ws (attn_bwd_fp8_ws_bytes), then the pass
int64_t attn_bwd_fp8_ws_bytes(int B, int N, int H);
void attn_bwd_dkdv8_launch(int dt, const void* qkv, const void* dout, const float* lse, const float* delta,
                           const float* nlse, const float* ndelta, void* dqkv, int B, int N, int H, float dk_scale,
                           float* r0q, void* f8ws, hipStream_t st);
// the one-pass backward (attention_bwd1.hip, DCLIP_OPT_ATTN_BWD_BLOCK 9): prep + sweep + ordered dQ
// reduction (the CLS row's merge is the caller's); r0kv gets attn_bwd1_prep_blocks(N) partials per
// (image, head), r0q one per key block; dqpart holds attn_bwd1_part_bytes
int attn_bwd1_prep_blocks(int N);
int64_t attn_bwd1_part_bytes(int B, int N, int H);
void attn_bwd1_launch(int dt, const void* qkv, const void* o, const void* dout, const float* lse, float* delta,
                      float* nstat, float* ds0v, float* r0kv, float* r0q, void* dqpart, void* dqkv, int B, int N,
                      int H, float scale, hipStream_t st);
