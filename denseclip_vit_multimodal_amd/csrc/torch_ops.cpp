// TORCH_LIBRARY(dclip) — the PyTorch-ROCm custom-op surface of the DenseCLIP ViT hot path
// (SURVEY §8(b) "Native ABI"): at::Tensor in, at::Tensor out, outputs allocated through the
// caching allocator, every launch on the current HIP stream of the input's device, errors as
// TORCH_CHECK (RuntimeError in Python; the reference's blanket try/except -> None of
// denseclip.py:733-752 is deliberately not reproduced).  Each op is a thin adapter over one
// entry point of the C ABI in include/dclip.h (libdclip.so), which cites the reference call it
// replaces.  No op synchronises with the host, so any op sequence can be captured in a
// hipGraph (torch.cuda.graph).  Fake (meta) implementations and autograd live in Python
// (denseclip_vit_multimodal_amd/ops.py: torch.library.register_fake, autograd.Function).
#include <ATen/ATen.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include "../../include/dclip.h"

namespace {

using at::Tensor;

int dt_code(at::ScalarType t) {
    switch (t) {
        case at::kFloat: return DCLIP_F32;
        case at::kHalf: return DCLIP_F16;
        case at::kBFloat16: return DCLIP_BF16;
        default: TORCH_CHECK(false, "dclip: unsupported dtype ", t);
    }
    return -1;
}

void* stream_of(const Tensor& t) { return (void*)c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

void check_gpu(const Tensor& t, const char* what, bool contiguous = true) {
    TORCH_CHECK(t.defined(), "dclip: ", what, " is undefined");
    TORCH_CHECK(t.is_cuda(), "dclip: ", what, " must be a GPU tensor (the MI355X path has no CPU fallback)");
    if (contiguous) TORCH_CHECK(t.is_contiguous(), "dclip: ", what, " must be contiguous");
}

void check_opt(const c10::optional<Tensor>& t, const char* what) {
    if (t.has_value() && t->defined()) check_gpu(*t, what);
}

// an optional per-column / per-channel f32 vector the kernels index [0, n): GPU, contiguous, f32, n elements
void check_vec(const c10::optional<Tensor>& t, int64_t n, const char* what) {
    if (!t.has_value() || !t->defined()) return;
    check_gpu(*t, what);
    TORCH_CHECK(t->scalar_type() == at::kFloat, "dclip: ", what, " must be float32 (got ", t->scalar_type(), ")");
    TORCH_CHECK(t->numel() == n, "dclip: ", what, " must have ", n, " elements (got ", t->numel(), ")");
}

template <typename T>
T* ptr(const Tensor& t) { return t.defined() ? (T*)t.data_ptr() : nullptr; }

template <typename T>
T* optr(const c10::optional<Tensor>& t) { return t.has_value() && t->defined() ? (T*)t->data_ptr() : nullptr; }

// entry i of a grad_scale() buffer (s, 1/s, 0, 0) on the op's device, or null without one
const float* scale_entry(const c10::optional<Tensor>& t, int i) {
    if (!t.has_value() || !t->defined()) return nullptr;
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->numel() == 4 && t->is_contiguous(),
                "scale must be a grad_scale() result: 4 contiguous f32 on the GPU");
    return (const float*)t->data_ptr() + i;
}

#define DCLIP_CALL(expr)                                                                    \
    do {                                                                                    \
        const int rc_ = (expr);                                                             \
        TORCH_CHECK(rc_ == 0, "dclip: ", #expr " failed (", rc_, "): ", dclip_last_error()); \
    } while (0)

at::TensorOptions like(const Tensor& t, at::ScalarType dt) { return t.options().dtype(dt); }

// ----------------------------------------------------------------------------- LayerNorm
// the LN backward's per-workgroup dw / db partials: private scratch of the call from the caching
// allocator (stream-ordered), or none when the pass has no dw / db or the width has no table
Tensor ln_ws(const Tensor& x, const Tensor& dw, const Tensor& db) {
    const int64_t n = (dw.defined() || db.defined()) ? dclip_layernorm_bwd_ws_floats(x.size(0), x.size(1)) : 0;
    return n > 0 ? at::empty({n}, like(x, at::kFloat)) : Tensor();
}

std::tuple<Tensor, Tensor, Tensor> layernorm_fwd(const Tensor& x, const Tensor& w, const Tensor& b,
                                                 at::ScalarType out_dtype, double eps) {
    check_gpu(x, "x"); check_gpu(w, "w"); check_gpu(b, "b");
    TORCH_CHECK(x.dim() == 2, "layernorm_fwd: x (rows, cols)");
    check_vec(w, x.size(1), "LayerNorm weight"); check_vec(b, x.size(1), "LayerNorm bias");
    c10::DeviceGuard g(x.device());
    const int64_t rows = x.size(0), cols = x.size(1);
    Tensor y = at::empty({rows, cols}, like(x, out_dtype));
    Tensor mean = at::empty({rows}, like(x, at::kFloat)), rstd = at::empty({rows}, like(x, at::kFloat));
    DCLIP_CALL(dclip_layernorm_fwd(x.data_ptr(), dt_code(x.scalar_type()), ptr<float>(w), ptr<float>(b), y.data_ptr(),
                                   dt_code(out_dtype), ptr<float>(mean), ptr<float>(rstd), rows, cols, (float)eps,
                                   stream_of(x)));
    return {y, mean, rstd};
}

// dx = res + LN^T(dy) (res optional); dw / db accumulated in place
// dy_scale: a (s, 1/s, ..) buffer whose 1/s multiplies dy on load (dy left on its gradient scale);
// dy_ntok > 0: dy's rows with row % dy_ntok == 0 (CLS) read as 0
Tensor layernorm_bwd(const Tensor& dy, const Tensor& x, const Tensor& w, const Tensor& mean, const Tensor& rstd,
                     const c10::optional<Tensor>& res, Tensor& dw, Tensor& db, const c10::optional<Tensor>& dy_scale,
                     int64_t dy_ntok) {
    check_gpu(dy, "dy"); check_gpu(x, "x"); check_gpu(w, "w"); check_gpu(mean, "mean"); check_gpu(rstd, "rstd");
    check_opt(res, "res"); check_opt(dy_scale, "dy_scale");
    TORCH_CHECK(x.dim() == 2 && dy.sizes() == x.sizes(), "layernorm_bwd: dy and x (rows, cols)");
    check_vec(w, x.size(1), "LayerNorm weight"); check_vec(dw, x.size(1), "dw"); check_vec(db, x.size(1), "db");
    check_vec(mean, x.size(0), "mean"); check_vec(rstd, x.size(0), "rstd");
    c10::DeviceGuard g(x.device());
    Tensor dx = at::empty(x.sizes(), like(x, at::kFloat));
    Tensor ws = ln_ws(x, dw, db);
    DCLIP_CALL(dclip_layernorm_bwd_res(dy.data_ptr(), dt_code(dy.scalar_type()), scale_entry(dy_scale, 1), dy_ntok,
                                       x.data_ptr(), dt_code(x.scalar_type()), ptr<float>(w), ptr<float>(mean),
                                       ptr<float>(rstd), optr<float>(res), ptr<float>(dx), nullptr, 0, ptr<float>(dw),
                                       ptr<float>(db), ptr<float>(ws), x.size(0), x.size(1), stream_of(x)));
    return dx;
}

// the same plus lp = (lp_dtype) dx, the next GEMM's 16-bit operand
std::tuple<Tensor, Tensor> layernorm_bwd_lp(const Tensor& dy, const Tensor& x, const Tensor& w, const Tensor& mean,
                                            const Tensor& rstd, const c10::optional<Tensor>& res, Tensor& dw,
                                            Tensor& db, at::ScalarType lp_dtype, const c10::optional<Tensor>& dy_scale) {
    check_gpu(dy, "dy"); check_gpu(x, "x"); check_gpu(w, "w"); check_gpu(mean, "mean"); check_gpu(rstd, "rstd");
    check_opt(res, "res"); check_opt(dy_scale, "dy_scale");
    TORCH_CHECK(x.dim() == 2 && dy.sizes() == x.sizes(), "layernorm_bwd: dy and x (rows, cols)");
    check_vec(w, x.size(1), "LayerNorm weight"); check_vec(dw, x.size(1), "dw"); check_vec(db, x.size(1), "db");
    check_vec(mean, x.size(0), "mean"); check_vec(rstd, x.size(0), "rstd");
    c10::DeviceGuard g(x.device());
    Tensor dx = at::empty(x.sizes(), like(x, at::kFloat));
    Tensor lp = at::empty(x.sizes(), like(x, lp_dtype));
    Tensor ws = ln_ws(x, dw, db);
    DCLIP_CALL(dclip_layernorm_bwd_res(dy.data_ptr(), dt_code(dy.scalar_type()), scale_entry(dy_scale, 1), 0,
                                       x.data_ptr(), dt_code(x.scalar_type()), ptr<float>(w), ptr<float>(mean),
                                       ptr<float>(rstd), optr<float>(res), ptr<float>(dx), lp.data_ptr(), dt_code(lp_dtype),
                                       ptr<float>(dw), ptr<float>(db), ptr<float>(ws), x.size(0), x.size(1),
                                       stream_of(x)));
    return {dx, lp};
}

// layernorm_bwd_lp of a block's ln_1 with the previous block's read-out map gradient `add` (bf16,
// rows with row % ntok == 0 read as 0) added before the cast: (dx, lp)
std::tuple<Tensor, Tensor> layernorm_bwd_add(const Tensor& dy, const Tensor& x, const Tensor& w, const Tensor& mean,
                                             const Tensor& rstd, const c10::optional<Tensor>& res, const Tensor& add,
                                             int64_t ntok, Tensor& dw, Tensor& db, at::ScalarType lp_dtype) {
    check_gpu(dy, "dy"); check_gpu(x, "x"); check_gpu(w, "w"); check_gpu(mean, "mean"); check_gpu(rstd, "rstd");
    check_gpu(add, "add"); check_opt(res, "res");
    TORCH_CHECK(x.dim() == 2 && dy.sizes() == x.sizes() && add.sizes() == x.sizes(),
                "layernorm_bwd_add: dy, x and add (rows, cols)");
    TORCH_CHECK(x.scalar_type() == at::kFloat && add.scalar_type() == at::kBFloat16,
                "layernorm_bwd_add: f32 x and a bf16 add buffer");
    TORCH_CHECK(ntok > 0 && x.size(0) % ntok == 0, "layernorm_bwd_add: rows must be a multiple of ntok");
    check_vec(w, x.size(1), "LayerNorm weight"); check_vec(dw, x.size(1), "dw"); check_vec(db, x.size(1), "db");
    check_vec(mean, x.size(0), "mean"); check_vec(rstd, x.size(0), "rstd");
    c10::DeviceGuard g(x.device());
    Tensor dx = at::empty(x.sizes(), like(x, at::kFloat));
    Tensor lp = at::empty(x.sizes(), like(x, lp_dtype));
    Tensor ws = ln_ws(x, dw, db);
    DCLIP_CALL(dclip_layernorm_bwd_add(dy.data_ptr(), dt_code(dy.scalar_type()), ptr<float>(x), ptr<float>(w),
                                       ptr<float>(mean), ptr<float>(rstd), optr<float>(res), add.data_ptr(), (int)ntok,
                                       ptr<float>(dx), lp.data_ptr(), dt_code(lp_dtype), ptr<float>(dw), ptr<float>(db),
                                       ptr<float>(ws), x.size(0), x.size(1), stream_of(x)));
    return {dx, lp};
}

// ----------------------------------------------------------------------------- GEMM
void gemm_checks(const Tensor& A, const Tensor& B) {
    TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.size(1) == B.size(1), "gemm: A (M, K), B (N, K)");
    TORCH_CHECK(A.stride(1) == 1 && B.stride(1) == 1, "gemm: operands must be k-contiguous");
    TORCH_CHECK(A.is_cuda() && B.is_cuda(), "gemm: GPU tensors only");
    TORCH_CHECK(A.scalar_type() == B.scalar_type(), "gemm: A and B dtypes differ");
}

// out[m][n] = alpha * sum_k A[m][k] B[n][k] (+ epilogue epi != GELU)
Tensor gemm(const Tensor& A, const Tensor& B, int64_t epi, const c10::optional<Tensor>& bias,
            const c10::optional<Tensor>& aux, at::ScalarType out_dtype, double alpha,
            const c10::optional<Tensor>& scale) {
    gemm_checks(A, B);
    TORCH_CHECK(epi != DCLIP_EPI_GELU && epi != DCLIP_EPI_SPLITK, "gemm: use gemm_gelu / weight_grad for this epilogue");
    TORCH_CHECK(epi >= DCLIP_EPI_STORE && epi <= DCLIP_EPI_STORE_SCALED, "gemm: unknown epilogue ", epi);
    c10::DeviceGuard g(A.device());
    const int64_t M = A.size(0), N = B.size(0), K = A.size(1);
    check_vec(bias, N, "gemm bias");
    const bool has_aux = aux.has_value() && aux->defined();
    if (has_aux) TORCH_CHECK(aux->is_cuda() && aux->stride(-1) == 1, "gemm: aux must be a row-major GPU tensor");
    if (epi == DCLIP_EPI_RESIDUAL || epi == DCLIP_EPI_GELU_BWD) {
        // the residual (f32) / the saved pre-activation z (A's dtype), read at [m][n]
        TORCH_CHECK(has_aux && aux->dim() == 2 && aux->size(0) == M && aux->size(1) == N,
                    "gemm: this epilogue needs aux of shape (M, N) = (", M, ", ", N, ")");
        TORCH_CHECK(epi != DCLIP_EPI_RESIDUAL || (aux->scalar_type() == at::kFloat && out_dtype == at::kFloat),
                    "gemm: the residual epilogue reads and writes float32");
        TORCH_CHECK(epi != DCLIP_EPI_GELU_BWD || aux->scalar_type() == A.scalar_type(),
                    "gemm: the QuickGELU' epilogue's aux (z) must have A's dtype");
    } else if (epi == DCLIP_EPI_STORE_SCALED) {
        TORCH_CHECK(has_aux, "gemm: the scaled epilogue needs the per-column scale aux");
        check_vec(aux, N, "gemm per-column scale (aux)");
    }
    Tensor out = at::empty({M, N}, like(A, out_dtype));
    DCLIP_CALL(dclip_gemm((int)epi, dt_code(A.scalar_type()), A.data_ptr(), A.stride(0), B.data_ptr(), B.stride(0), M, N,
                          K, 1, (float)alpha, scale_entry(scale, 1), optr<float>(bias),
                          has_aux ? aux->data_ptr() : nullptr,
                          has_aux ? dt_code(aux->scalar_type()) : 0, has_aux && aux->dim() == 2 ? aux->stride(0) : 0,
                          out.data_ptr(), dt_code(out_dtype), out.stride(0), nullptr, 0, stream_of(A)));
    return out;
}

// out = aux + A B^T + bias (f32 residual epilogue) and lp = (A's dtype) out in the same epilogue:
// the new residual stream and its 16-bit copy (a per-layer read-out map's token buffer,
// models.py:577-582) without a separate cast pass
std::tuple<Tensor, Tensor> gemm_residual_lp(const Tensor& A, const Tensor& B, const c10::optional<Tensor>& bias,
                                            const Tensor& aux) {
    gemm_checks(A, B);
    c10::DeviceGuard g(A.device());
    const int64_t M = A.size(0), N = B.size(0), K = A.size(1);
    check_vec(bias, N, "gemm_residual_lp bias");
    check_gpu(aux, "aux", false);
    TORCH_CHECK(aux.dim() == 2 && aux.size(0) == M && aux.size(1) == N && aux.stride(1) == 1 &&
                    aux.scalar_type() == at::kFloat,
                "gemm_residual_lp: aux must be the f32 (M, N) residual");
    Tensor out = at::empty({M, N}, like(A, at::kFloat)), lp = at::empty({M, N}, A.options());
    DCLIP_CALL(dclip_gemm(DCLIP_EPI_RESIDUAL, dt_code(A.scalar_type()), A.data_ptr(), A.stride(0), B.data_ptr(),
                          B.stride(0), M, N, K, 1, 1.0f, nullptr, optr<float>(bias), aux.data_ptr(), DCLIP_F32,
                          aux.stride(0), out.data_ptr(), DCLIP_F32, out.stride(0), lp.data_ptr(), lp.stride(0),
                          stream_of(A)));
    return {out, lp};
}

// z = A B^T + bias, h = quick_gelu(z)  (c_fc + QuickGELU, models.py:277-281, 252-254)
std::tuple<Tensor, Tensor> gemm_gelu(const Tensor& A, const Tensor& B, const c10::optional<Tensor>& bias) {
    gemm_checks(A, B);
    c10::DeviceGuard g(A.device());
    const int64_t M = A.size(0), N = B.size(0), K = A.size(1);
    check_vec(bias, N, "gemm_gelu bias");
    Tensor z = at::empty({M, N}, A.options()), h = at::empty({M, N}, A.options());
    DCLIP_CALL(dclip_gemm(DCLIP_EPI_GELU, dt_code(A.scalar_type()), A.data_ptr(), A.stride(0), B.data_ptr(), B.stride(0),
                          M, N, K, 1, 1.0f, nullptr, optr<float>(bias), nullptr, 0, 0, z.data_ptr(), dt_code(A.scalar_type()),
                          z.stride(0), h.data_ptr(), h.stride(0), stream_of(A)));
    return {z, h};
}

// inference form: h = quick_gelu(x W^T + b) only (no z for a backward)
Tensor gemm_gelu_h(const Tensor& A, const Tensor& B, const c10::optional<Tensor>& bias) {
    gemm_checks(A, B);
    c10::DeviceGuard g(A.device());
    const int64_t M = A.size(0), N = B.size(0), K = A.size(1);
    check_vec(bias, N, "gemm_gelu_h bias");
    Tensor h = at::empty({M, N}, A.options());
    DCLIP_CALL(dclip_gemm(DCLIP_EPI_GELU, dt_code(A.scalar_type()), A.data_ptr(), A.stride(0), B.data_ptr(), B.stride(0),
                          M, N, K, 1, 1.0f, nullptr, optr<float>(bias), nullptr, 0, 0, nullptr, dt_code(A.scalar_type()),
                          N, h.data_ptr(), h.stride(0), stream_of(A)));
    return h;
}

// dW = alpha dy^T x (f32) and, when db is given, db += alpha colsum(dy)
Tensor weight_grad(const Tensor& dy, const Tensor& x, double alpha, c10::optional<Tensor> db,
                   const c10::optional<Tensor>& scale) {
    check_gpu(dy, "dy"); check_gpu(x, "x");
    TORCH_CHECK(dy.dim() == 2 && x.dim() == 2 && dy.size(0) == x.size(0), "weight_grad: dy (M, N), x (M, K)");
    TORCH_CHECK(dy.scalar_type() == x.scalar_type(), "weight_grad: dy and x dtypes differ (", dy.scalar_type(), " vs ",
                x.scalar_type(), ")");
    c10::DeviceGuard g(dy.device());
    const int64_t M = dy.size(0), N = dy.size(1), K = x.size(1);
    check_vec(db, N, "weight_grad db");
    int splits = 0;
    int64_t k_pad = 0;
    DCLIP_CALL(dclip_gemm_tn_plan(N, K, M, &splits, &k_pad));
    Tensor dW = at::empty({N, K}, like(dy, at::kFloat));
    Tensor ws = at::empty({(int64_t)splits * (N * K + N)}, like(dy, at::kFloat));
    DCLIP_CALL(dclip_gemm_tn(DCLIP_EPI_SPLITK, dt_code(dy.scalar_type()), dy.data_ptr(), dy.stride(0), x.data_ptr(),
                             x.stride(0), N, K, M, k_pad, splits, (float)alpha, scale_entry(scale, 1), nullptr, ws.data_ptr(),
                             dW.data_ptr(), K,
                             optr<float>(db), stream_of(dy)));
    return dW;
}

// out[m][n] = sum_k A[k][m] B[k][n] (f32)
Tensor gemm_tn(const Tensor& A, const Tensor& B) {
    check_gpu(A, "A"); check_gpu(B, "B");
    TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.size(0) == B.size(0), "gemm_tn: A (K, M), B (K, N)");
    c10::DeviceGuard g(A.device());
    const int64_t K = A.size(0), M = A.size(1), N = B.size(1);
    Tensor out = at::empty({M, N}, like(A, at::kFloat));
    DCLIP_CALL(dclip_gemm_tn(DCLIP_EPI_STORE, dt_code(A.scalar_type()), A.data_ptr(), A.stride(0), B.data_ptr(),
                             B.stride(0), M, N, K, (K + 63) / 64 * 64, 1, 1.0f, nullptr, nullptr, nullptr, out.data_ptr(), N,
                             nullptr, stream_of(A)));
    return out;
}

// ----------------------------------------------------------------------------- element-wise
// (s, 1/s, 0, 0) f32 on the device: the power-of-two fp16 scale of the gradient g (dclip_grad_scale)
Tensor grad_scale(const Tensor& g, double target) {
    check_gpu(g, "g");
    TORCH_CHECK(g.scalar_type() == at::kFloat && g.is_contiguous(), "grad_scale: g must be contiguous f32");
    c10::DeviceGuard gd(g.device());
    Tensor ws = at::zeros({4}, g.options());
    DCLIP_CALL(dclip_grad_scale(ptr<float>(g), g.numel(), (float)target, ptr<float>(ws), stream_of(g)));
    return ws;
}

Tensor cast(const Tensor& x, at::ScalarType dtype, double scale, const c10::optional<Tensor>& scale_t) {
    check_gpu(x, "x");
    c10::DeviceGuard g(x.device());
    Tensor y = at::empty(x.sizes(), like(x, dtype));
    DCLIP_CALL(dclip_cast(x.data_ptr(), dt_code(x.scalar_type()), y.data_ptr(), dt_code(dtype), x.numel(), (float)scale,
                          scale_entry(scale_t, 0), stream_of(x)));
    return y;
}

// 2-D transpose (rows, cols) -> (cols, rows) in dtype
Tensor transpose2d(const Tensor& x, at::ScalarType dtype) {
    check_gpu(x, "x");
    TORCH_CHECK(x.dim() == 2, "transpose2d: 2-D input");
    c10::DeviceGuard g(x.device());
    const int64_t rows = x.size(0), cols = x.size(1);
    Tensor out = at::empty({cols, rows}, like(x, dtype));
    DCLIP_CALL(dclip_transpose(x.data_ptr(), dt_code(x.scalar_type()), 0, cols, 0, out.data_ptr(), dt_code(dtype),
                               cols * rows, rows, 1, rows, rows, cols, 0, nullptr, stream_of(x)));
    return out;
}

// every cached compute-dtype copy of the stepped weights rewritten in one launch (C ABI
// dclip_weight_refresh): desc = the (n, 8) int64 descriptor on the weights' device (built and
// cached by ops.refresh_weight_copies); writes only through the pointers it holds
void weight_refresh(const Tensor& desc, int64_t tiles, at::ScalarType dtype) {
    check_gpu(desc, "desc");
    TORCH_CHECK(desc.scalar_type() == at::kLong && desc.dim() == 2 && desc.size(1) == 8,
                "weight_refresh: desc must be an (n, 8) int64 tensor");
    c10::DeviceGuard g(desc.device());
    DCLIP_CALL(dclip_weight_refresh((const int64_t*)desc.data_ptr(), (int)desc.size(0), tiles, dt_code(dtype),
                                    stream_of(desc)));
}

// out[b][c][r] = x[b][r][c] for r < rows, c < cols (x rows of ld_in elements, batch stride
// rows*ld_in); r in [rows, rows_pad) written as zeros: (B, cols, rows_pad) in dtype
Tensor transpose_batched(const Tensor& x, int64_t B, int64_t rows, int64_t cols, int64_t ld_in, int64_t rows_pad,
                         at::ScalarType dtype) {
    check_gpu(x, "x");
    TORCH_CHECK(x.numel() >= B * rows * ld_in && cols <= ld_in && rows_pad >= rows, "transpose_batched: shapes");
    c10::DeviceGuard g(x.device());
    Tensor out = at::empty({B, cols, rows_pad}, like(x, dtype));
    DCLIP_CALL(dclip_transpose(x.data_ptr(), dt_code(x.scalar_type()), rows * ld_in, ld_in, 0, out.data_ptr(),
                               dt_code(dtype), cols * rows_pad, rows_pad, (int)B, rows, rows_pad, cols, 0, nullptr,
                               stream_of(x)));
    return out;
}

std::tuple<Tensor, Tensor> add_readout_cast(const Tensor& a, const Tensor& b, int64_t ntok, at::ScalarType lp_dtype,
                                            double scale) {
    check_gpu(a, "a"); check_gpu(b, "b", false);
    TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && b.stride(1) == 1 && b.stride(0) == a.size(1) && a.sizes() == b.sizes(),
                "add_readout_cast: a, b (rows, cols) row-major");
    c10::DeviceGuard g(a.device());
    Tensor sum = at::empty(a.sizes(), a.options());
    Tensor lp = at::empty(a.sizes(), like(a, lp_dtype));
    DCLIP_CALL(dclip_add_readout_cast(ptr<float>(a), b.data_ptr(), dt_code(b.scalar_type()), ptr<float>(sum), lp.data_ptr(),
                                      dt_code(lp_dtype), a.size(0), (int)a.size(1), (int)ntok, (float)scale, stream_of(a)));
    return {sum, lp};
}

// fp16 form: (a + b * 1/s_heads with b's CLS rows masked, the grad_scale() pair of that sum)
std::tuple<Tensor, Tensor> add_readout_amax(const Tensor& a, const Tensor& b, int64_t ntok,
                                            const c10::optional<Tensor>& b_scale, double target) {
    check_gpu(a, "a"); check_gpu(b, "b", false);
    TORCH_CHECK(a.scalar_type() == at::kFloat, "add_readout_amax: a must be f32");
    TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && b.stride(1) == 1 && b.stride(0) == a.size(1) && a.sizes() == b.sizes(),
                "add_readout_amax: a, b (rows, cols) row-major");
    c10::DeviceGuard g(a.device());
    Tensor sum = at::empty(a.sizes(), a.options());
    Tensor ws = at::zeros({4}, a.options());
    DCLIP_CALL(dclip_add_readout_amax(ptr<float>(a), b.data_ptr(), dt_code(b.scalar_type()), scale_entry(b_scale, 1),
                                      ptr<float>(sum), a.size(0), (int)a.size(1), (int)ntok, (float)target,
                                      ptr<float>(ws), stream_of(a)));
    return {sum, ws};
}

// delayed-scale state of one fp16 gradient site: DCLIP_DS_STATE_FLOATS contiguous f32 on the op's device
float* scale_state(const Tensor& st, const Tensor& like_t) {
    TORCH_CHECK(st.is_cuda() && st.scalar_type() == at::kFloat && st.numel() == DCLIP_DS_STATE_FLOATS &&
                    st.is_contiguous() && st.device() == like_t.device(),
                "scale state must be DCLIP_DS_STATE_FLOATS contiguous f32 on the op's GPU");
    return (float*)st.data_ptr();
}

// fp16 delayed-scale form: (sum = a + b * 1/s_heads (b's CLS rows masked; no b: an empty tensor, the sum is a),
// lp = (f16)(sum * s_state), the (s, 1/s) pair lp was cast with); st advanced to this use's scale
std::tuple<Tensor, Tensor, Tensor> add_readout_cast_scaled(const Tensor& a, const c10::optional<Tensor>& b, int64_t ntok,
                                                           const c10::optional<Tensor>& b_scale, Tensor& st, int64_t use, double target) {
    check_gpu(a, "a");
    const bool has_b = b.has_value() && b->defined();
    TORCH_CHECK(a.scalar_type() == at::kFloat && a.dim() == 2 && a.numel() > 0, "add_readout_cast_scaled: a (rows, cols) f32");
    if (has_b) {
        check_gpu(*b, "b", false);
        TORCH_CHECK(b->dim() == 2 && b->stride(1) == 1 && b->stride(0) == a.size(1) && a.sizes() == b->sizes(),
                    "add_readout_cast_scaled: a, b (rows, cols) row-major");
    }
    c10::DeviceGuard g(a.device());
    Tensor sum = has_b ? at::empty(a.sizes(), a.options()) : at::empty({0}, a.options());  // no b: sum is a
    Tensor lp = at::empty(a.sizes(), like(a, at::kHalf));
    Tensor pair = at::empty({4}, a.options());
    DCLIP_CALL(dclip_add_readout_cast_scaled(ptr<float>(a), has_b ? b->data_ptr() : nullptr,
                                             has_b ? dt_code(b->scalar_type()) : DCLIP_F32, scale_entry(b_scale, 1),
                                             has_b ? ptr<float>(sum) : nullptr, lp.data_ptr(), a.size(0), (int)a.size(1),
                                             (int)ntok, (float)target, scale_state(st, a), (int)use, ptr<float>(pair),
                                             stream_of(a)));
    return {sum, lp, pair};
}

// layernorm_bwd_lp with an fp16 lp cast on the delayed scale of st: (dx, lp, the (s, 1/s) pair)
std::tuple<Tensor, Tensor, Tensor> layernorm_bwd_scaled(const Tensor& dy, const Tensor& x, const Tensor& w,
                                                        const Tensor& mean, const Tensor& rstd,
                                                        const c10::optional<Tensor>& res, Tensor& dw, Tensor& db,
                                                        Tensor& st, int64_t use, double target,
                                                        const c10::optional<Tensor>& dy_scale) {
    check_gpu(dy, "dy"); check_gpu(x, "x"); check_gpu(w, "w"); check_gpu(mean, "mean"); check_gpu(rstd, "rstd");
    check_opt(res, "res"); check_opt(dy_scale, "dy_scale");
    TORCH_CHECK(x.dim() == 2 && dy.sizes() == x.sizes() && x.size(0) > 0, "layernorm_bwd_scaled: dy and x (rows, cols)");
    TORCH_CHECK((dy.scalar_type() == at::kFloat || dy.scalar_type() == at::kHalf) && x.scalar_type() == at::kFloat,
                "layernorm_bwd_scaled: f32 or f16 dy, f32 x");
    check_vec(w, x.size(1), "LayerNorm weight"); check_vec(dw, x.size(1), "dw"); check_vec(db, x.size(1), "db");
    check_vec(mean, x.size(0), "mean"); check_vec(rstd, x.size(0), "rstd");
    c10::DeviceGuard g(x.device());
    Tensor dx = at::empty(x.sizes(), like(x, at::kFloat));
    Tensor lp = at::empty(x.sizes(), like(x, at::kHalf));
    Tensor pair = at::empty({4}, x.options());
    Tensor ws = ln_ws(x, dw, db);
    DCLIP_CALL(dclip_layernorm_bwd_scaled(dy.data_ptr(), dt_code(dy.scalar_type()), scale_entry(dy_scale, 1), x.data_ptr(),
                                          dt_code(x.scalar_type()), ptr<float>(w), ptr<float>(mean), ptr<float>(rstd),
                                          optr<float>(res), ptr<float>(dx),
                                          lp.data_ptr(), ptr<float>(dw), ptr<float>(db), ptr<float>(ws), x.size(0), x.size(1),
                                          (float)target, scale_state(st, x), (int)use, ptr<float>(pair), stream_of(x)));
    return {dx, lp, pair};
}

// layernorm_bwd_scaled with the previous block's read-out map gradient `add` (16-bit, CLS rows read
// as 0) times add_scale[1] (a HeadScale (s, 1/s, ..) buffer: the heads' 1/s; optional) added before
// the delayed-scale fp16 cast
std::tuple<Tensor, Tensor, Tensor> layernorm_bwd_scaled_add(const Tensor& dy, const Tensor& x, const Tensor& w,
                                                            const Tensor& mean, const Tensor& rstd,
                                                            const c10::optional<Tensor>& res, const Tensor& add,
                                                            const c10::optional<Tensor>& add_scale, int64_t ntok,
                                                            Tensor& dw, Tensor& db, Tensor& st, int64_t use,
                                                            double target, const c10::optional<Tensor>& dy_scale) {
    check_gpu(dy, "dy"); check_gpu(x, "x"); check_gpu(w, "w"); check_gpu(mean, "mean"); check_gpu(rstd, "rstd");
    check_gpu(add, "add"); check_opt(res, "res"); check_opt(add_scale, "add_scale"); check_opt(dy_scale, "dy_scale");
    TORCH_CHECK(x.dim() == 2 && dy.sizes() == x.sizes() && add.sizes() == x.sizes() && x.size(0) > 0,
                "layernorm_bwd_scaled_add: dy, x and add (rows, cols)");
    TORCH_CHECK((dy.scalar_type() == at::kFloat || dy.scalar_type() == at::kHalf) && x.scalar_type() == at::kFloat &&
                    (add.scalar_type() == at::kHalf || add.scalar_type() == at::kBFloat16),
                "layernorm_bwd_scaled_add: f32 or f16 dy, f32 x, a 16-bit add buffer");
    TORCH_CHECK(ntok > 0 && x.size(0) % ntok == 0, "layernorm_bwd_scaled_add: rows must be a multiple of ntok");
    check_vec(w, x.size(1), "LayerNorm weight"); check_vec(dw, x.size(1), "dw"); check_vec(db, x.size(1), "db");
    check_vec(mean, x.size(0), "mean"); check_vec(rstd, x.size(0), "rstd");
    c10::DeviceGuard g(x.device());
    Tensor dx = at::empty(x.sizes(), like(x, at::kFloat));
    Tensor lp = at::empty(x.sizes(), like(x, at::kHalf));
    Tensor pair = at::empty({4}, x.options());
    Tensor ws = ln_ws(x, dw, db);
    DCLIP_CALL(dclip_layernorm_bwd_scaled_add(dy.data_ptr(), dt_code(dy.scalar_type()), scale_entry(dy_scale, 1),
                                              ptr<float>(x), ptr<float>(w), ptr<float>(mean),
                                              ptr<float>(rstd), optr<float>(res), add.data_ptr(),
                                              dt_code(add.scalar_type()), scale_entry(add_scale, 1), (int)ntok,
                                              ptr<float>(dx), lp.data_ptr(), ptr<float>(dw), ptr<float>(db),
                                              ptr<float>(ws), x.size(0),
                                              x.size(1), (float)target, scale_state(st, x), (int)use, ptr<float>(pair),
                                              stream_of(x)));
    return {dx, lp, pair};
}

// (x ? x : 0) + s[row % ntok] * y, f32 (rows, cols): a drop_path-scaled residual branch
Tensor row_scale_add(const c10::optional<Tensor>& x, const Tensor& y, const Tensor& s) {
    check_gpu(y, "y"); check_gpu(s, "s"); check_opt(x, "x");
    TORCH_CHECK(y.scalar_type() == at::kFloat && s.scalar_type() == at::kFloat && y.dim() == 2,
                "row_scale_add: y (rows, cols) f32, s (ntok,) f32");
    const bool has_x = x.has_value() && x->defined();
    if (has_x) TORCH_CHECK(x->scalar_type() == at::kFloat && x->sizes() == y.sizes(), "row_scale_add: x like y");
    c10::DeviceGuard g(y.device());
    Tensor out = at::empty(y.sizes(), y.options());
    DCLIP_CALL(dclip_row_scale_add(has_x ? ptr<float>(*x) : nullptr, ptr<float>(y), ptr<float>(s), (int)s.numel(),
                                   ptr<float>(out), y.size(0), (int)y.size(1), stream_of(y)));
    return out;
}

// ----------------------------------------------------------------------------- attention
std::tuple<Tensor, Tensor> attn_fwd(const Tensor& qkv, int64_t B, int64_t N, int64_t H, double scale) {
    check_gpu(qkv, "qkv");
    TORCH_CHECK(qkv.dim() == 2 && qkv.size(0) == B * N && qkv.size(1) == 3 * 64 * H, "attn_fwd: qkv (B*N, 3*H*64)");
    c10::DeviceGuard g(qkv.device());
    Tensor o = at::empty({B * N, 64 * H}, qkv.options());
    Tensor lse = at::empty({B * H * N}, like(qkv, at::kFloat));
    DCLIP_CALL(dclip_attn_fwd(dt_code(qkv.scalar_type()), qkv.data_ptr(), o.data_ptr(), ptr<float>(lse), (int)B, (int)N,
                              (int)H, 64, (float)scale, stream_of(qkv)));
    return {o, lse};
}

std::tuple<Tensor, Tensor> attn_fwd_fp8(const Tensor& qkv, int64_t B, int64_t N, int64_t H) {
    check_gpu(qkv, "qkv");
    TORCH_CHECK(qkv.dim() == 2 && qkv.size(0) == B * N && qkv.size(1) == 3 * 64 * H, "attn_fwd_fp8: qkv (B*N, 3*H*64)");
    c10::DeviceGuard g(qkv.device());
    Tensor o = at::empty({B * N, 64 * H}, qkv.options());
    Tensor lse = at::empty({B * H * N}, like(qkv, at::kFloat));
    Tensor ws = at::empty({dclip_attn_fwd_fp8_workspace((int)B, (int)N, (int)H)}, like(qkv, at::kByte));
    DCLIP_CALL(dclip_attn_fwd_fp8(dt_code(qkv.scalar_type()), qkv.data_ptr(), o.data_ptr(), ptr<float>(lse), ws.data_ptr(),
                                  (int)B, (int)N, (int)H, 64, stream_of(qkv)));
    return {o, lse};
}

Tensor attn_bwd(const Tensor& qkv, const Tensor& o, const Tensor& dout, const Tensor& lse, int64_t B, int64_t N,
                int64_t H, double scale) {
    check_gpu(qkv, "qkv"); check_gpu(o, "o"); check_gpu(dout, "dout"); check_gpu(lse, "lse");
    TORCH_CHECK(qkv.size(0) == B * N && o.sizes() == dout.sizes() && o.size(1) == 64 * H, "attn_bwd: shapes");
    c10::DeviceGuard g(qkv.device());
    Tensor ws = at::empty({dclip_attn_bwd_workspace((int)B, (int)N, (int)H)}, like(qkv, at::kFloat));
    Tensor dqkv = at::empty_like(qkv);
    DCLIP_CALL(dclip_attn_bwd(dt_code(qkv.scalar_type()), qkv.data_ptr(), o.data_ptr(), dout.data_ptr(), ptr<float>(lse),
                              ptr<float>(ws), dqkv.data_ptr(), (int)B, (int)N, (int)H, 64, (float)scale, stream_of(qkv)));
    return dqkv;
}

// configs[4]'s backward: dV, dK on the block-scaled e4m3 MFMA (dclip_attn_bwd_fp8)
Tensor attn_bwd_fp8(const Tensor& qkv, const Tensor& o, const Tensor& dout, const Tensor& lse, int64_t B, int64_t N,
                    int64_t H, double scale) {
    check_gpu(qkv, "qkv"); check_gpu(o, "o"); check_gpu(dout, "dout"); check_gpu(lse, "lse");
    TORCH_CHECK(qkv.size(0) == B * N && o.sizes() == dout.sizes() && o.size(1) == 64 * H, "attn_bwd_fp8: shapes");
    c10::DeviceGuard g(qkv.device());
    Tensor ws = at::empty({dclip_attn_bwd_fp8_workspace((int)B, (int)N, (int)H)}, like(qkv, at::kFloat));
    Tensor dqkv = at::empty_like(qkv);
    DCLIP_CALL(dclip_attn_bwd_fp8(dt_code(qkv.scalar_type()), qkv.data_ptr(), o.data_ptr(), dout.data_ptr(),
                                  ptr<float>(lse), ptr<float>(ws), dqkv.data_ptr(), (int)B, (int)N, (int)H, 64,
                                  (float)scale, stream_of(qkv)));
    return dqkv;
}

// ----------------------------------------------------------------------------- patch embedding
Tensor im2col(const Tensor& img, int64_t p, at::ScalarType dtype) {
    check_gpu(img, "img");
    TORCH_CHECK(img.dim() == 4, "im2col: img (B, Cin, H, W)");
    c10::DeviceGuard g(img.device());
    const int64_t B = img.size(0), Cin = img.size(1), Hin = img.size(2), Win = img.size(3);
    const int64_t k_pad = (Cin * p * p + 63) / 64 * 64;
    Tensor out = at::empty({B * (Hin / p) * (Win / p), k_pad}, like(img, dtype));
    DCLIP_CALL(dclip_im2col(img.data_ptr(), dt_code(img.scalar_type()), out.data_ptr(), dt_code(dtype), k_pad, (int)B,
                            (int)Cin, (int)Hin, (int)Win, (int)p, stream_of(img)));
    return out;
}

Tensor tokens_fwd(const Tensor& emb, const Tensor& cls, const Tensor& pos, int64_t B, int64_t P) {
    check_gpu(emb, "emb"); check_gpu(cls, "cls"); check_gpu(pos, "pos");
    const int64_t C = emb.size(1);
    TORCH_CHECK(emb.size(0) == B * P && pos.size(0) == P + 1 && cls.numel() == C, "tokens_fwd: shapes");
    c10::DeviceGuard g(emb.device());
    Tensor x = at::empty({B * (P + 1), C}, like(emb, at::kFloat));
    DCLIP_CALL(dclip_tokens_fwd(emb.data_ptr(), dt_code(emb.scalar_type()), ptr<float>(cls), ptr<float>(pos), ptr<float>(x),
                                (int)B, (int)P, (int)C, stream_of(emb)));
    return x;
}

// (demb = scale * dx[patch rows] in dtype, dcls, dpos (P+1, C))
std::tuple<Tensor, Tensor, Tensor> tokens_bwd(const Tensor& dx, at::ScalarType dtype, double scale, int64_t B,
                                              int64_t P, const c10::optional<Tensor>& scale_t) {
    check_gpu(dx, "dx");
    const int64_t C = dx.size(1);
    TORCH_CHECK(dx.size(0) == B * (P + 1), "tokens_bwd: dx (B*(P+1), C)");
    c10::DeviceGuard g(dx.device());
    Tensor demb = at::empty({B * P, C}, like(dx, dtype));
    Tensor dcls = at::zeros({C}, like(dx, at::kFloat));
    Tensor dpos = at::zeros({P + 1, C}, like(dx, at::kFloat));
    DCLIP_CALL(dclip_tokens_bwd(ptr<float>(dx), demb.data_ptr(), dt_code(dtype), (float)scale,
                                scale_entry(scale_t, 0), ptr<float>(dcls),
                                ptr<float>(dpos), (int)B, (int)P, (int)C, stream_of(dx)));
    return {demb, dcls, dpos};
}

Tensor pos_interp(const Tensor& pos, int64_t g, int64_t H, int64_t W) {
    check_gpu(pos, "pos");
    TORCH_CHECK(pos.scalar_type() == at::kFloat && pos.size(0) == g * g + 1, "pos_interp: pos (g*g+1, C) fp32");
    c10::DeviceGuard gd(pos.device());
    Tensor out = at::empty({H * W + 1, pos.size(1)}, pos.options());
    DCLIP_CALL(dclip_pos_interp_fwd(ptr<float>(pos), ptr<float>(out), (int)g, (int)pos.size(1), (int)H, (int)W,
                                    stream_of(pos)));
    return out;
}

Tensor pos_interp_bwd(const Tensor& dout, int64_t g, int64_t H, int64_t W) {
    check_gpu(dout, "dout");
    TORCH_CHECK(dout.scalar_type() == at::kFloat && dout.size(0) == H * W + 1, "pos_interp_bwd: dout (H*W+1, C) fp32");
    c10::DeviceGuard gd(dout.device());
    Tensor dpos = at::zeros({g * g + 1, dout.size(1)}, dout.options());
    DCLIP_CALL(dclip_pos_interp_bwd(ptr<float>(dout), ptr<float>(dpos), (int)g, (int)dout.size(1), (int)H, (int)W,
                                    stream_of(dout)));
    return dpos;
}

// ----------------------------------------------------------------------------- score map / resize
// strided pixel rows (dclip.h): row r of image b at x + b*bstride + (row_off + r)*ld (elements)
void check_rows(const Tensor& x, int64_t bstride, int64_t row_off, int64_t ld, int64_t B, int64_t rows, int64_t C) {
    TORCH_CHECK(x.is_cuda() && x.stride(-1) == 1, "dclip: pixel rows must be a GPU tensor with unit column stride");
    const int64_t last = (B - 1) * bstride + (row_off + rows - 1) * ld + C;  // one past the last element read
    TORCH_CHECK(x.storage_offset() + last <= (int64_t)(x.storage().nbytes() / x.element_size()),
                "dclip: the strided rows run past the tensor's storage");
}

Tensor row_mean(const Tensor& x, int64_t bstride, int64_t row_off, int64_t ld, int64_t B, int64_t rows, int64_t C) {
    check_rows(x, bstride, row_off, ld, B, rows, C);
    c10::DeviceGuard g(x.device());
    Tensor ws = at::empty({dclip_row_mean_workspace((int)B, rows, (int)C)}, like(x, at::kFloat));
    Tensor out = at::empty({B, C}, like(x, at::kFloat));
    DCLIP_CALL(dclip_row_mean(x.data_ptr(), dt_code(x.scalar_type()), bstride, row_off, ld, (int)B, rows, (int)C,
                              ptr<float>(ws), ptr<float>(out), stream_of(x)));
    return out;
}

Tensor score_map(const Tensor& v, int64_t bstride, int64_t row_off, int64_t ld, const Tensor& text, int64_t B,
                 int64_t HW, double eps) {
    check_gpu(text, "text");
    TORCH_CHECK(text.scalar_type() == at::kFloat && text.dim() == 3 && text.size(0) == B, "score_map: text (B, K, C) fp32");
    const int64_t K = text.size(1), C = text.size(2);
    check_rows(v, bstride, row_off, ld, B, HW, C);
    c10::DeviceGuard g(v.device());
    Tensor out = at::empty({B, K, HW}, like(v, at::kFloat));
    DCLIP_CALL(dclip_score_map(v.data_ptr(), dt_code(v.scalar_type()), bstride, row_off, ld, ptr<float>(text),
                               ptr<float>(out), (int)B, (int)HW, (int)C, (int)K, (float)eps, stream_of(v)));
    return out;
}

// (B*h*w, C+K) channels-last rows: the C strided pixel-row channels of a read-out map, then the K
// channels of the f32 score (B, K, hs, ws) bilinearly resized to (h, w)
Tensor score_concat(const Tensor& rows, int64_t bstride, int64_t row_off, int64_t ld, int64_t C, const Tensor& score,
                    int64_t B, int64_t h, int64_t w) {
    check_gpu(score, "score");
    TORCH_CHECK(score.scalar_type() == at::kFloat && score.dim() == 4 && score.size(0) == B,
                "score_concat: score (B, K, hs, ws) fp32");
    check_rows(rows, bstride, row_off, ld, B, h * w, C);
    c10::DeviceGuard g(rows.device());
    const int64_t K = score.size(1);
    Tensor out = at::empty({B * h * w, C + K}, rows.options());
    DCLIP_CALL(dclip_score_concat(rows.data_ptr(), dt_code(rows.scalar_type()), bstride, row_off, ld, (int)C,
                                  ptr<float>(score), (int)K, (int)score.size(2), (int)score.size(3), out.data_ptr(),
                                  (int)B, (int)h, (int)w, stream_of(rows)));
    return out;
}

Tensor bilinear(const Tensor& x, int64_t Ho, int64_t Wo, at::ScalarType dtype) {
    check_gpu(x, "x");
    TORCH_CHECK(x.dim() == 4, "bilinear: x (n, c, h, w)");
    c10::DeviceGuard g(x.device());
    Tensor out = at::empty({x.size(0), x.size(1), Ho, Wo}, like(x, dtype));
    DCLIP_CALL(dclip_bilinear_fwd(x.data_ptr(), dt_code(x.scalar_type()), out.data_ptr(), dt_code(dtype),
                                  x.size(0) * x.size(1), (int)x.size(2), (int)x.size(3), (int)Ho, (int)Wo, stream_of(x)));
    return out;
}

Tensor bilinear_bwd(const Tensor& dout, int64_t Hi, int64_t Wi) {
    check_gpu(dout, "dout");
    TORCH_CHECK(dout.dim() == 4, "bilinear_bwd: dout (n, c, H, W)");
    c10::DeviceGuard g(dout.device());
    const int64_t nc = dout.size(0) * dout.size(1), Ho = dout.size(2), Wo = dout.size(3);
    Tensor din = at::empty({dout.size(0), dout.size(1), Hi, Wi}, like(dout, at::kFloat));
    Tensor ws = at::empty({nc * Ho * Wi}, like(dout, at::kFloat));
    DCLIP_CALL(dclip_bilinear_bwd(dout.data_ptr(), dt_code(dout.scalar_type()), ptr<float>(din), ptr<float>(ws), nc,
                                  (int)Hi, (int)Wi, (int)Ho, (int)Wo, stream_of(dout)));
    return din;
}

// ----------------------------------------------------------------------------- BatchNorm (+ ReLU), train mode
// rows view of a map: a channels-last 4-D tensor (pitch C) or a 2-D (rows, C) view with unit column
// stride (a channel slice of a wider buffer: pitch = stride(0))
struct Rows {
    int64_t rows, C, ld;
};

Rows rows_of(const Tensor& x) {
    TORCH_CHECK(x.is_cuda(), "dclip: BatchNorm input must be a GPU tensor");
    if (x.dim() == 4) {
        TORCH_CHECK(x.is_contiguous(at::MemoryFormat::ChannelsLast), "dclip: BatchNorm map must be channels-last");
        return {x.numel() / x.size(1), x.size(1), x.size(1)};
    }
    TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1, "dclip: BatchNorm rows must be 2-D with unit column stride");
    return {x.size(0), x.size(1), x.stride(0)};
}

std::tuple<Tensor, Tensor> bn_fwd_into(const Tensor& x, const c10::optional<Tensor>& w, const c10::optional<Tensor>& b,
                                       const c10::optional<Tensor>& running_mean, const c10::optional<Tensor>& running_var,
                                       double momentum, double eps, bool relu, const Tensor& y) {
    const Rows r = rows_of(x), ry = rows_of(y);
    TORCH_CHECK(r.rows == ry.rows && r.C == ry.C && r.ld == ry.ld && x.scalar_type() == y.scalar_type(),
                "dclip: BatchNorm output must match the input's rows, channels and pitch");
    check_vec(w, r.C, "BatchNorm weight"); check_vec(b, r.C, "BatchNorm bias");
    check_vec(running_mean, r.C, "running_mean"); check_vec(running_var, r.C, "running_var");
    c10::DeviceGuard g(x.device());
    Tensor ws = at::empty({dclip_bn_workspace(r.rows, (int)r.C)}, like(x, at::kFloat));
    Tensor mean = at::empty({r.C}, like(x, at::kFloat)), rstd = at::empty({r.C}, like(x, at::kFloat));
    DCLIP_CALL(dclip_bn_fwd(dt_code(x.scalar_type()), x.data_ptr(), r.rows, (int)r.C, r.ld, optr<float>(w), optr<float>(b),
                            (float)eps, (float)momentum, optr<float>(running_mean), optr<float>(running_var),
                            ptr<float>(ws), ptr<float>(mean), ptr<float>(rstd), y.data_ptr(), relu ? 1 : 0, stream_of(x)));
    return {mean, rstd};
}

std::tuple<Tensor, Tensor, Tensor> bn_fwd(const Tensor& x, const c10::optional<Tensor>& w,
                                          const c10::optional<Tensor>& b, const c10::optional<Tensor>& running_mean,
                                          const c10::optional<Tensor>& running_var, double momentum, double eps,
                                          bool relu) {
    TORCH_CHECK(x.dim() == 4, "bn_fwd: a channels-last 4-D map");
    Tensor y = at::empty_like(x, at::MemoryFormat::ChannelsLast);
    auto ms = bn_fwd_into(x, w, b, running_mean, running_var, momentum, eps, relu, y);
    return {y, std::get<0>(ms), std::get<1>(ms)};
}

// eval mode (running statistics), channels-last map in, channels-last map out
Tensor bn_eval(const Tensor& x, const c10::optional<Tensor>& w, const c10::optional<Tensor>& b,
               const Tensor& running_mean, const Tensor& running_var, double eps, bool relu) {
    TORCH_CHECK(x.dim() == 4, "bn_eval: a channels-last 4-D map");
    const Rows r = rows_of(x);
    check_vec(w, r.C, "BatchNorm weight"); check_vec(b, r.C, "BatchNorm bias");
    check_vec(running_mean, r.C, "running_mean"); check_vec(running_var, r.C, "running_var");
    c10::DeviceGuard g(x.device());
    Tensor y = at::empty_like(x, at::MemoryFormat::ChannelsLast);
    Tensor ws = at::empty({dclip_bn_workspace(r.rows, (int)r.C)}, like(x, at::kFloat));
    DCLIP_CALL(dclip_bn_eval(dt_code(x.scalar_type()), x.data_ptr(), r.rows, (int)r.C, r.ld, optr<float>(w),
                             optr<float>(b), (float)eps, ptr<float>(running_mean), ptr<float>(running_var),
                             ptr<float>(ws), y.data_ptr(), relu ? 1 : 0, stream_of(x)));
    return y;
}

// (rows view) y written in place into the caller's buffer
std::tuple<Tensor, Tensor> bn_fwd_rows(const Tensor& x, const c10::optional<Tensor>& w, const c10::optional<Tensor>& b,
                                       c10::optional<Tensor> running_mean, c10::optional<Tensor> running_var,
                                       double momentum, double eps, bool relu, Tensor& y) {
    return bn_fwd_into(x, w, b, running_mean, running_var, momentum, eps, relu, y);
}

std::tuple<Tensor, Tensor> bn_bwd_into(const Tensor& dy, const Tensor& x, const c10::optional<Tensor>& w,
                                       const c10::optional<Tensor>& b, const Tensor& mean, const Tensor& rstd, bool relu,
                                       bool want_w, bool want_b, const Tensor& dx,
                                       const c10::optional<Tensor>& scale = c10::nullopt) {
    const Rows r = rows_of(x), rd = rows_of(dy), rdx = rows_of(dx);
    TORCH_CHECK(rd.rows == r.rows && rd.C == r.C && rd.ld == r.ld && rdx.ld == r.ld && rdx.rows == r.rows,
                "dclip: BatchNorm backward tensors must share rows, channels and pitch");
    TORCH_CHECK(dy.scalar_type() == x.scalar_type() && dx.scalar_type() == x.scalar_type(), "bn_bwd: dtypes must match");
    check_vec(w, r.C, "BatchNorm weight"); check_vec(b, r.C, "BatchNorm bias");
    check_vec(mean, r.C, "mean"); check_vec(rstd, r.C, "rstd");
    c10::DeviceGuard g(x.device());
    Tensor ws = at::empty({dclip_bn_workspace(r.rows, (int)r.C)}, like(x, at::kFloat));
    Tensor dw = want_w ? at::empty({r.C}, like(x, at::kFloat)) : at::empty({0}, like(x, at::kFloat));
    Tensor db = want_b ? at::empty({r.C}, like(x, at::kFloat)) : at::empty({0}, like(x, at::kFloat));
    DCLIP_CALL(dclip_bn_bwd(dt_code(x.scalar_type()), dy.data_ptr(), x.data_ptr(), r.rows, (int)r.C, r.ld, optr<float>(w),
                            optr<float>(b), ptr<float>(mean), ptr<float>(rstd), ptr<float>(ws), dx.data_ptr(),
                            want_w ? ptr<float>(dw) : nullptr, want_b ? ptr<float>(db) : nullptr, relu ? 1 : 0,
                            scale_entry(scale, 1), stream_of(x)));
    return {dw, db};
}

std::tuple<Tensor, Tensor, Tensor> bn_bwd(const Tensor& dy, const Tensor& x, const c10::optional<Tensor>& w,
                                          const c10::optional<Tensor>& b, const Tensor& mean, const Tensor& rstd,
                                          bool relu, bool want_w, bool want_b, const c10::optional<Tensor>& scale) {
    TORCH_CHECK(x.dim() == 4, "bn_bwd: a channels-last 4-D map");
    Tensor dx = at::empty_like(x, at::MemoryFormat::ChannelsLast);
    auto g = bn_bwd_into(dy, x, w, b, mean, rstd, relu, want_w, want_b, dx, scale);
    return {dx, std::get<0>(g), std::get<1>(g)};
}

std::tuple<Tensor, Tensor> bn_bwd_rows(const Tensor& dy, const Tensor& x, const c10::optional<Tensor>& w,
                                       const c10::optional<Tensor>& b, const Tensor& mean, const Tensor& rstd, bool relu,
                                       bool want_w, bool want_b, Tensor& dx, const c10::optional<Tensor>& scale) {
    return bn_bwd_into(dy, x, w, b, mean, rstd, relu, want_w, want_b, dx, scale);
}

// ----------------------------------------------------------------------------- neck 3x3 conv
// X: any GPU tensor whose data_ptr is input pixel (0, 0, 0) (a channels-last map or a token-
// buffer view); geometry in elements as in dclip.h.  out: written (or accumulated) in place.
void conv3x3(int64_t mode, const Tensor& X, int64_t x_bstride, int64_t x_off, int64_t x_ld, int64_t B, int64_t H,
             int64_t W, int64_t Cin, const Tensor& Wt, int64_t Nout, Tensor& out, int64_t out_ld, int64_t out_gap,
             int64_t out_off, int64_t accumulate) {
    check_gpu(X, "X", false); check_gpu(Wt, "Wt"); check_gpu(out, "out", false);
    TORCH_CHECK(X.scalar_type() == Wt.scalar_type(), "conv3x3: X and Wt dtypes differ");
    c10::DeviceGuard g(X.device());
    DCLIP_CALL(dclip_conv3x3((int)mode, dt_code(X.scalar_type()), X.data_ptr(), x_bstride, x_off, x_ld, (int)B, (int)H,
                             (int)W, (int)Cin, Wt.data_ptr(), (int)Nout, out.data_ptr(), dt_code(out.scalar_type()), out_ld,
                             (int)out_gap, (int)out_off, (int)accumulate, stream_of(X)));
}

Tensor conv3x3_wgrad(const Tensor& dY, int64_t ldy, int64_t Nout, const Tensor& X, int64_t x_bstride, int64_t x_off,
                     int64_t x_ld, int64_t B, int64_t H, int64_t W, int64_t Cin, int64_t splits, bool oihw,
                     const c10::optional<Tensor>& scale) {
    check_gpu(dY, "dY", false); check_gpu(X, "X", false);
    TORCH_CHECK(oihw || !(scale.has_value() && scale->defined()), "conv3x3_wgrad: a scale needs the OIHW output");
    c10::DeviceGuard g(X.device());
    Tensor dW = oihw ? at::empty({Nout, Cin, 3, 3}, like(X, at::kFloat)) : at::empty({Nout, 9 * Cin}, like(X, at::kFloat));
    Tensor ws = at::empty({splits * Nout * 9 * Cin}, like(X, at::kFloat));
    DCLIP_CALL(dclip_conv3x3_wgrad(dt_code(dY.scalar_type()), dY.data_ptr(), ldy, (int)Nout, X.data_ptr(), x_bstride,
                                   x_off, x_ld, (int)B, (int)H, (int)W, (int)Cin, ptr<float>(dW), ws.data_ptr(),
                                   (int)splits, oihw ? 1 : 0, scale_entry(scale, 1), stream_of(X)));
    return dW;
}

// ----------------------------------------------------------------------------- fused head losses
int lab_code(at::ScalarType t) {
    switch (t) {
        case at::kLong: return 0;
        case at::kInt: return 1;
        case at::kByte: return 2;
        default: TORCH_CHECK(false, "upsample_ce: labels must be int64, int32 or uint8");
    }
    return -1;
}

// (loss sum f64[1], valid count i32[1], un-normalised low-res gradient f32)
std::tuple<Tensor, Tensor, Tensor> upsample_ce(const Tensor& logits, const Tensor& labels, int64_t ignore_index) {
    check_gpu(logits, "logits"); check_gpu(labels, "labels");
    TORCH_CHECK(logits.dim() == 4 && labels.dim() == 3 && labels.size(0) == logits.size(0), "upsample_ce: shapes");
    c10::DeviceGuard g(logits.device());
    Tensor sums = at::zeros({1}, like(logits, at::kDouble));
    Tensor cnt = at::zeros({1}, like(logits, at::kInt));
    Tensor grad = at::zeros(logits.sizes(), like(logits, at::kFloat));
    Tensor ws = at::empty({dclip_upsample_ws_floats((int)logits.size(0), (int)logits.size(1), (int)logits.size(2),
                                                    (int)logits.size(3))}, like(logits, at::kFloat));
    DCLIP_CALL(dclip_upsample_ce(dt_code(logits.scalar_type()), logits.data_ptr(), (int)logits.size(0),
                                 (int)logits.size(1), (int)logits.size(2), (int)logits.size(3), labels.data_ptr(),
                                 lab_code(labels.scalar_type()), (int)labels.size(1), (int)labels.size(2),
                                 (int)ignore_index, (double*)sums.data_ptr(), (unsigned*)cnt.data_ptr(), ptr<float>(grad),
                                 ptr<float>(ws), stream_of(logits)));
    return {sums, cnt, grad};
}

// pass 0 of the SILog pair: sums f64[3] = (sum d, sum d^2, T)
Tensor upsample_silog_sums(const Tensor& pred, const Tensor& target, const c10::optional<Tensor>& mask, double eps) {
    check_gpu(pred, "pred"); check_gpu(target, "target"); check_opt(mask, "mask");
    TORCH_CHECK(target.scalar_type() == at::kFloat && target.dim() == 3, "upsample_silog: target (B, H, W) fp32");
    c10::DeviceGuard g(pred.device());
    Tensor sums = at::zeros({3}, like(pred, at::kDouble));
    Tensor ws = at::empty({dclip_upsample_ws_floats((int)pred.size(0), 1, (int)pred.size(2), (int)pred.size(3))},
                          like(pred, at::kFloat));
    DCLIP_CALL(dclip_upsample_silog(0, dt_code(pred.scalar_type()), pred.data_ptr(), (int)pred.size(0), (int)pred.size(2),
                                    (int)pred.size(3), ptr<float>(target), optr<uint8_t>(mask), (int)target.size(1),
                                    (int)target.size(2), (float)eps, 0.f, (double*)sums.data_ptr(), nullptr,
                                    ptr<float>(ws), stream_of(pred)));
    return sums;
}

// pass 1: d loss / d pred (low-res, f32) from the complete sums
Tensor upsample_silog_grad(const Tensor& pred, const Tensor& target, const c10::optional<Tensor>& mask,
                           const Tensor& sums, double eps, double lambd) {
    check_gpu(pred, "pred"); check_gpu(target, "target"); check_opt(mask, "mask"); check_gpu(sums, "sums");
    c10::DeviceGuard g(pred.device());
    Tensor grad = at::zeros(pred.sizes(), like(pred, at::kFloat));
    Tensor ws = at::empty({dclip_upsample_ws_floats((int)pred.size(0), 1, (int)pred.size(2), (int)pred.size(3))},
                          like(pred, at::kFloat));
    DCLIP_CALL(dclip_upsample_silog(1, dt_code(pred.scalar_type()), pred.data_ptr(), (int)pred.size(0), (int)pred.size(2),
                                    (int)pred.size(3), ptr<float>(target), optr<uint8_t>(mask), (int)target.size(1),
                                    (int)target.size(2), (float)eps, (float)lambd, (double*)sums.data_ptr(),
                                    ptr<float>(grad), ptr<float>(ws), stream_of(pred)));
    return grad;
}

// ----------------------------------------------------------------------------- Cityscapes batch preparation
std::tuple<Tensor, Tensor, Tensor, Tensor> cityscapes_prepare(const Tensor& img, const Tensor& ids, const Tensor& disp,
                                                              const Tensor& crop, int64_t h, int64_t w,
                                                              at::ArrayRef<double> mean, at::ArrayRef<double> stdv,
                                                              double bf, double depth_max, at::ScalarType out_dtype,
                                                              const c10::optional<Tensor>& jitter) {
    check_gpu(img, "img"); check_gpu(ids, "ids"); check_gpu(disp, "disp"); check_gpu(crop, "crop");
    TORCH_CHECK(mean.size() == 3 && stdv.size() == 3, "cityscapes_prepare: 3 means / stds");
    TORCH_CHECK(img.dim() == 4 && img.size(3) == 3 && crop.scalar_type() == at::kInt, "cityscapes_prepare: shapes");
    // crop (B, 3) = window + flip; crop (B, 7) = the RandomScale / PadIfNeeded parameters in front
    const bool aug = crop.dim() == 2 && crop.size(1) == 7;
    TORCH_CHECK(crop.dim() == 2 && (crop.size(1) == 3 || aug) && crop.size(0) == img.size(0),
                "cityscapes_prepare: crop (B, 3) or params (B, 7) int32");
    c10::DeviceGuard g(img.device());
    const int64_t B = img.size(0), H = img.size(1), W = img.size(2);
    Tensor out_img = at::empty({B, 3, h, w}, like(img, out_dtype));
    Tensor seg = at::empty({B, h, w}, like(img, at::kLong));
    Tensor depth = at::empty({B, 1, h, w}, like(img, at::kFloat));
    Tensor mask = at::empty({B, 1, h, w}, like(img, at::kByte));
    const float m[3] = {(float)mean[0], (float)mean[1], (float)mean[2]};
    const float s[3] = {(float)stdv[0], (float)stdv[1], (float)stdv[2]};
    const bool jit = jitter.has_value() && jitter->defined();
    if (jit) {
        // ColorJitter sits between the spatial transforms and Normalize: the crop as uint8 HWC, the
        // jitter in place, then the normalisation
        TORCH_CHECK(aug, "cityscapes_prepare: ColorJitter needs the (B, 7) scale / pad / crop parameters");
        TORCH_CHECK(jitter->is_cuda() && jitter->scalar_type() == at::kDouble && jitter->dim() == 2 &&
                        jitter->size(0) == B && jitter->size(1) == 8 && jitter->is_contiguous(),
                    "cityscapes_prepare: jitter must be (B, 8) float64 on the GPU");
        Tensor u8 = at::empty({B, h, w, 3}, like(img, at::kByte));
        Tensor ws = at::empty({B}, like(img, at::kLong));
        DCLIP_CALL(dclip_cityscapes_augment(ptr<uint8_t>(img), ptr<uint8_t>(ids), (const uint16_t*)disp.data_ptr(),
                                            (int)B, (int)H, (int)W, ptr<int>(crop), (int)h, (int)w, m, s, (float)bf,
                                            (float)depth_max, u8.data_ptr(), DCLIP_U8, ptr<int64_t>(seg),
                                            ptr<float>(depth), ptr<uint8_t>(mask), stream_of(img)));
        DCLIP_CALL(dclip_color_jitter(ptr<uint8_t>(u8), (int)B, (int)h, (int)w, (const double*)jitter->data_ptr(),
                                      (unsigned long long*)ws.data_ptr(), stream_of(img)));
        DCLIP_CALL(dclip_normalize_u8(ptr<uint8_t>(u8), (int)B, (int)h, (int)w, m, s, out_img.data_ptr(),
                                      dt_code(out_dtype), stream_of(img)));
        return {out_img, seg, depth, mask};
    }
    auto fn = aug ? &dclip_cityscapes_augment : &dclip_cityscapes_prepare;
    DCLIP_CALL(fn(ptr<uint8_t>(img), ptr<uint8_t>(ids), (const uint16_t*)disp.data_ptr(), (int)B, (int)H, (int)W,
                  ptr<int>(crop), (int)h, (int)w, m, s, (float)bf, (float)depth_max, out_img.data_ptr(),
                  dt_code(out_dtype), ptr<int64_t>(seg), ptr<float>(depth), ptr<uint8_t>(mask), stream_of(img)));
    return {out_img, seg, depth, mask};
}

}  // namespace

TORCH_LIBRARY(dclip, m) {
    m.def("layernorm_fwd(Tensor x, Tensor w, Tensor b, ScalarType out_dtype, float eps) -> (Tensor, Tensor, Tensor)");
    m.def("layernorm_bwd(Tensor dy, Tensor x, Tensor w, Tensor mean, Tensor rstd, Tensor? res, Tensor(a!) dw, "
          "Tensor(b!) db, Tensor? dy_scale=None, int dy_ntok=0) -> Tensor");
    m.def("layernorm_bwd_lp(Tensor dy, Tensor x, Tensor w, Tensor mean, Tensor rstd, Tensor? res, Tensor(a!) dw, "
          "Tensor(b!) db, ScalarType lp_dtype, Tensor? dy_scale=None) -> (Tensor, Tensor)");
    m.def("layernorm_bwd_add(Tensor dy, Tensor x, Tensor w, Tensor mean, Tensor rstd, Tensor? res, Tensor add, "
          "int ntok, Tensor(a!) dw, Tensor(b!) db, ScalarType lp_dtype) -> (Tensor, Tensor)");
    m.def("gemm(Tensor A, Tensor B, int epi, Tensor? bias, Tensor? aux, ScalarType out_dtype, float alpha, "
          "Tensor? scale=None) -> Tensor");
    m.def("gemm_gelu(Tensor A, Tensor B, Tensor? bias) -> (Tensor, Tensor)");
    m.def("gemm_gelu_h(Tensor A, Tensor B, Tensor? bias) -> Tensor");
    m.def("gemm_residual_lp(Tensor A, Tensor B, Tensor? bias, Tensor aux) -> (Tensor, Tensor)");
    m.def("weight_grad(Tensor dy, Tensor x, float alpha, Tensor(a!)? db, Tensor? scale=None) -> Tensor");
    m.def("gemm_tn(Tensor A, Tensor B) -> Tensor");
    m.def("cast(Tensor x, ScalarType dtype, float scale, Tensor? scale_t=None) -> Tensor");
    m.def("grad_scale(Tensor g, float target) -> Tensor");
    m.def("row_scale_add(Tensor? x, Tensor y, Tensor s) -> Tensor");
    m.def("bn_eval(Tensor x, Tensor? w, Tensor? b, Tensor running_mean, Tensor running_var, float eps, bool relu) -> Tensor");
    m.def("transpose2d(Tensor x, ScalarType dtype) -> Tensor");
    m.def("weight_refresh(Tensor desc, int tiles, ScalarType dtype) -> ()");
    m.def("transpose_batched(Tensor x, int B, int rows, int cols, int ld_in, int rows_pad, ScalarType dtype) -> Tensor");
    m.def("add_readout_cast(Tensor a, Tensor b, int ntok, ScalarType lp_dtype, float scale) -> (Tensor, Tensor)");
    m.def("add_readout_amax(Tensor a, Tensor b, int ntok, Tensor? b_scale, float target) -> (Tensor, Tensor)");
    m.def("add_readout_cast_scaled(Tensor a, Tensor? b, int ntok, Tensor? b_scale, Tensor(a!) st, int use, float target) "
          "-> (Tensor, Tensor, Tensor)");
    m.def("layernorm_bwd_scaled(Tensor dy, Tensor x, Tensor w, Tensor mean, Tensor rstd, Tensor? res, Tensor(a!) dw, "
          "Tensor(b!) db, Tensor(c!) st, int use, float target, Tensor? dy_scale=None) -> (Tensor, Tensor, Tensor)");
    m.def("layernorm_bwd_scaled_add(Tensor dy, Tensor x, Tensor w, Tensor mean, Tensor rstd, Tensor? res, "
          "Tensor add, Tensor? add_scale, int ntok, Tensor(a!) dw, Tensor(b!) db, Tensor(c!) st, int use, "
          "float target, Tensor? dy_scale=None) -> (Tensor, Tensor, Tensor)");
    m.def("attn_fwd(Tensor qkv, int B, int N, int H, float scale) -> (Tensor, Tensor)");
    m.def("attn_fwd_fp8(Tensor qkv, int B, int N, int H) -> (Tensor, Tensor)");
    m.def("attn_bwd(Tensor qkv, Tensor o, Tensor dout, Tensor lse, int B, int N, int H, float scale) -> Tensor");
    m.def("attn_bwd_fp8(Tensor qkv, Tensor o, Tensor dout, Tensor lse, int B, int N, int H, float scale) -> Tensor");
    m.def("im2col(Tensor img, int p, ScalarType dtype) -> Tensor");
    m.def("tokens_fwd(Tensor emb, Tensor cls, Tensor pos, int B, int P) -> Tensor");
    m.def("tokens_bwd(Tensor dx, ScalarType dtype, float scale, int B, int P, Tensor? scale_t=None) -> "
          "(Tensor, Tensor, Tensor)");
    m.def("pos_interp(Tensor pos, int g, int H, int W) -> Tensor");
    m.def("pos_interp_bwd(Tensor dout, int g, int H, int W) -> Tensor");
    m.def("row_mean(Tensor x, int bstride, int row_off, int ld, int B, int rows, int C) -> Tensor");
    m.def("score_map(Tensor v, int bstride, int row_off, int ld, Tensor text, int B, int HW, float eps) -> Tensor");
    m.def("score_concat(Tensor rows, int bstride, int row_off, int ld, int C, Tensor score, int B, int h, int w) -> Tensor");
    m.def("bilinear(Tensor x, int Ho, int Wo, ScalarType dtype) -> Tensor");
    m.def("bilinear_bwd(Tensor dout, int Hi, int Wi) -> Tensor");
    m.def("bn_fwd(Tensor x, Tensor? w, Tensor? b, Tensor(a!)? running_mean, Tensor(b!)? running_var, float momentum, "
          "float eps, bool relu) -> (Tensor, Tensor, Tensor)");
    m.def("bn_bwd(Tensor dy, Tensor x, Tensor? w, Tensor? b, Tensor mean, Tensor rstd, bool relu, bool want_w, "
          "bool want_b, Tensor? scale=None) -> (Tensor, Tensor, Tensor)");
    m.def("bn_fwd_rows(Tensor x, Tensor? w, Tensor? b, Tensor(a!)? running_mean, Tensor(b!)? running_var, "
          "float momentum, float eps, bool relu, Tensor(c!) y) -> (Tensor, Tensor)");
    m.def("bn_bwd_rows(Tensor dy, Tensor x, Tensor? w, Tensor? b, Tensor mean, Tensor rstd, bool relu, bool want_w, "
          "bool want_b, Tensor(a!) dx, Tensor? scale=None) -> (Tensor, Tensor)");
    m.def("conv3x3(int mode, Tensor X, int x_bstride, int x_off, int x_ld, int B, int H, int W, int Cin, Tensor Wt, "
          "int Nout, Tensor(a!) out, int out_ld, int out_gap, int out_off, int accumulate) -> ()");
    m.def("conv3x3_wgrad(Tensor dY, int ldy, int Nout, Tensor X, int x_bstride, int x_off, int x_ld, int B, int H, "
          "int W, int Cin, int splits, bool oihw=False, Tensor? scale=None) -> Tensor");
    m.def("upsample_ce(Tensor logits, Tensor labels, int ignore_index) -> (Tensor, Tensor, Tensor)");
    m.def("upsample_silog_sums(Tensor pred, Tensor target, Tensor? mask, float eps) -> Tensor");
    m.def("upsample_silog_grad(Tensor pred, Tensor target, Tensor? mask, Tensor sums, float eps, float lambd) -> Tensor");
    m.def("cityscapes_prepare(Tensor img, Tensor ids, Tensor disp, Tensor crop, int h, int w, float[] mean, "
          "float[] std, float bf, float depth_max, ScalarType out_dtype, Tensor? jitter=None) -> "
          "(Tensor, Tensor, Tensor, Tensor)");
}

TORCH_LIBRARY_IMPL(dclip, CUDA, m) {
    m.impl("layernorm_fwd", &layernorm_fwd);
    m.impl("layernorm_bwd", &layernorm_bwd);
    m.impl("layernorm_bwd_lp", &layernorm_bwd_lp);
    m.impl("layernorm_bwd_add", &layernorm_bwd_add);
    m.impl("gemm", &gemm);
    m.impl("gemm_gelu", &gemm_gelu);
    m.impl("gemm_gelu_h", &gemm_gelu_h);
    m.impl("gemm_residual_lp", &gemm_residual_lp);
    m.impl("weight_grad", &weight_grad);
    m.impl("gemm_tn", &gemm_tn);
    m.impl("cast", &cast);
    m.impl("grad_scale", &grad_scale);
    m.impl("row_scale_add", &row_scale_add);
    m.impl("bn_eval", &bn_eval);
    m.impl("transpose2d", &transpose2d);
    m.impl("weight_refresh", &weight_refresh);
    m.impl("transpose_batched", &transpose_batched);
    m.impl("add_readout_cast", &add_readout_cast);
    m.impl("add_readout_amax", &add_readout_amax);
    m.impl("add_readout_cast_scaled", &add_readout_cast_scaled);
    m.impl("layernorm_bwd_scaled", &layernorm_bwd_scaled);
    m.impl("layernorm_bwd_scaled_add", &layernorm_bwd_scaled_add);
    m.impl("attn_fwd", &attn_fwd);
    m.impl("attn_fwd_fp8", &attn_fwd_fp8);
    m.impl("attn_bwd", &attn_bwd);
    m.impl("attn_bwd_fp8", &attn_bwd_fp8);
    m.impl("im2col", &im2col);
    m.impl("tokens_fwd", &tokens_fwd);
    m.impl("tokens_bwd", &tokens_bwd);
    m.impl("pos_interp", &pos_interp);
    m.impl("pos_interp_bwd", &pos_interp_bwd);
    m.impl("row_mean", &row_mean);
    m.impl("score_map", &score_map);
    m.impl("score_concat", &score_concat);
    m.impl("bilinear", &bilinear);
    m.impl("bilinear_bwd", &bilinear_bwd);
    m.impl("bn_fwd", &bn_fwd);
    m.impl("bn_bwd", &bn_bwd);
    m.impl("bn_fwd_rows", &bn_fwd_rows);
    m.impl("bn_bwd_rows", &bn_bwd_rows);
    m.impl("conv3x3", &conv3x3);
    m.impl("conv3x3_wgrad", &conv3x3_wgrad);
    m.impl("upsample_ce", &upsample_ce);
    m.impl("upsample_silog_sums", &upsample_silog_sums);
    m.impl("upsample_silog_grad", &upsample_silog_grad);
    m.impl("cityscapes_prepare", &cityscapes_prepare);
}
