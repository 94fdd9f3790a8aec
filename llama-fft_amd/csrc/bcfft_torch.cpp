// C++ torch operators over the C ABI (include/bcfft.h): torch.ops.bcfft_native.forward and
// forward_glu. The hot call of bcfft.ops.forward / forward_glu without the ctypes marshalling:
// argument checks, the output allocation, the split-K workspace and the stream lookup happen in
// C++ behind one dispatcher call. Host code only (the kernels are libbcfft.so's); a Meta kernel
// gives shapes and dtypes to FakeTensor / torch.compile tracing. Same checks, errors and
// semantics as the Python path (bcfft/ops.py), which stays as the fallback when this library is
// not built.
//   BlockCirculantLinear.forward: reference src/patch_llama_fft.py:226-275
//   fused gate/up + SwiGLU:        reference src/patch_llama_fft.py:343-394
#include <ATen/ATen.h>
#include <ATen/core/dispatch/Dispatcher.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <cstdint>
#include <optional>
#include <string>

#include "bcfft.h"

namespace {

int dtype_code(at::ScalarType t) {
  switch (t) {
    case at::kFloat: return BCFFT_F32;
    case at::kHalf: return BCFFT_F16;
    case at::kBFloat16: return BCFFT_BF16;
    default: TORCH_CHECK_TYPE(false, "unsupported dtype ", t, "; BC engine supports float32/float16/bfloat16");
  }
  return BCFFT_NONE;
}

void check_status(int st, const char* what) {
  if (st == BCFFT_OK) return;
  std::string msg = std::string(what) + " failed: " + bcfft_status_string(st);
  if (st == BCFFT_ERR_HIP) msg += std::string(" (") + bcfft_last_hip_error() + ")";
  if (st == BCFFT_ERR_BLOCK) {
    const char* d = bcfft_last_error_detail();
    if (d && *d) msg += std::string(" [") + d + "]";
  }
  TORCH_CHECK(false, msg);
}

void require_device(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda(), what, ": the MI355X BC engine runs on ROCm device tensors only (got ", t.device(),
              "); move the module and inputs to the GPU. There is no CPU path in the product.");
}

// 16-B aligned contiguous view (the kernels read x, bias and spectra with 16-B loads)
at::Tensor aligned(const at::Tensor& t) {
  at::Tensor c = t.contiguous();
  return reinterpret_cast<uintptr_t>(c.data_ptr()) % 16 ? c.clone() : c;
}

// the library cannot see the spectra buffer's size: a buffer built for another geometry would be
// read out of bounds (bcfft/ops.py _check_spectra)
void check_spectra(const at::Tensor& spec, int64_t n_out, int64_t n_in, int64_t b, const char* what) {
  TORCH_CHECK_VALUE(b > 0 && n_out > 0 && n_in > 0, what, ": invalid geometry (out_blocks=", n_out,
                    ", in_blocks=", n_in, ", block_size=", b, ")");
  const int64_t need = bcfft_spectra_bytes((int)n_out, (int)n_in, (int)b);
  TORCH_CHECK_VALUE(need >= 0 && spec.scalar_type() == at::kFloat && spec.numel() * 4 >= need, what,
                    ": spectra buffer of ", spec.numel() * spec.element_size(), " B (", spec.scalar_type(),
                    ") does not hold the (", n_out, ", ", n_in, ", ", b, ") operator (", need, " B)");
}

// a spectra buffer or bias read by raw pointer must live on x's device; a spectra buffer must be
// contiguous (the library indexes the flat packed image) (bcfft/ops.py _check_operand)
void check_operand(const at::Tensor& t, const at::Tensor& x, const char* what, const char* name, bool spectra) {
  TORCH_CHECK_VALUE(t.device() == x.device(), what, ": ", name, " is on ", t.device(), " but x is on ", x.device(),
                    "; move it to x's device");
  TORCH_CHECK_VALUE(!spectra || t.is_contiguous(), what,
                    ": the spectra buffer must be contiguous (use bcfft.ops.spectra's output as is)");
}

at::ScalarType out_dtype(const at::Tensor& x, const std::optional<at::Tensor>& bias) {
  return bias.has_value() ? at::promote_types(x.scalar_type(), bias->scalar_type()) : x.scalar_type();
}

at::Tensor forward_hip(const at::Tensor& x, const at::Tensor& spec, const std::optional<at::Tensor>& bias,
                       int64_t block_size, int64_t out_features, int64_t algo, bool split_k) {
  require_device(x, "bcfft.forward");
  TORCH_CHECK_VALUE(x.dim() == 2, "bcfft.forward: x2d must be (N, in_features)");
  const int64_t n = x.size(0), k = x.size(1);
  if (block_size > 0 && out_features % block_size == 0 && k % block_size == 0)
    check_spectra(spec, out_features / block_size, k / block_size, block_size, "bcfft.forward");
  check_operand(spec, x, "bcfft.forward", "spectra", true);
  if (bias.has_value()) check_operand(*bias, x, "bcfft.forward", "bias", false);
  const c10::DeviceGuard guard(x.device());
  const at::Tensor xa = aligned(x);
  at::Tensor y = at::empty({n, out_features}, x.options().dtype(out_dtype(x, bias)));
  if (n == 0) return y;
  at::Tensor ba;
  const void* bptr = nullptr;
  int bcode = BCFFT_NONE;
  if (bias.has_value()) {
    ba = aligned(bias->detach());
    bptr = ba.data_ptr();
    bcode = dtype_code(ba.scalar_type());
  }
  const int xc = dtype_code(xa.scalar_type()), yc = dtype_code(y.scalar_type());
  // split-K workspace (short grids of the MFMA and streamed-weight kernels) from torch's allocator;
  // the query is host logic keyed by the geometry, so a layer called again with the same shape
  // (every decode step, every prefill batch of one size) reuses the last answer. The answer depends
  // on the current device's CU count (split-K slices, the short-N rule), so the device is part of
  // the key: one thread driving GPUs of different sizes re-queries per device.
  struct WsKey {
    int64_t n, k, o, b, algo;
    int xc, yc, dev;
    bool operator==(const WsKey& r) const {
      return n == r.n && k == r.k && o == r.o && b == r.b && algo == r.algo && xc == r.xc && yc == r.yc &&
             dev == r.dev;
    }
  };
  thread_local WsKey ws_key{-1, 0, 0, 0, 0, 0, 0, -1};
  thread_local int64_t ws_cached = 0;
  int64_t ws_bytes = 0;
  if (split_k) {
    const WsKey key{n, k, out_features, block_size, algo, xc, yc, (int)x.device().index()};
    if (!(key == ws_key)) {
      ws_cached = bcfft_forward_workspace_bytes_io(n, (int)k, (int)out_features, (int)block_size, (int)algo, xc, yc);
      ws_key = key;
    }
    ws_bytes = ws_cached;
  }
  at::Tensor ws;
  if (ws_bytes > 0) ws = at::empty({ws_bytes}, x.options().dtype(at::kByte));
  else ws_bytes = 0;
  const hipStream_t s = c10::hip::getCurrentHIPStream(x.device().index()).stream();
  check_status(bcfft_forward_ws(xa.data_ptr(), xc, n, (int)k, (int)out_features, (int)block_size, spec.data_ptr(),
                                bptr, bcode, y.data_ptr(), yc, (int)algo, ws_bytes ? ws.data_ptr() : nullptr,
                                ws_bytes, s),
               "bcfft_forward");
  return y;
}

at::Tensor forward_meta(const at::Tensor& x, const at::Tensor& spec, const std::optional<at::Tensor>& bias,
                        int64_t block_size, int64_t out_features, int64_t algo, bool split_k) {
  TORCH_CHECK_VALUE(x.dim() == 2, "bcfft::forward: x2d must be (N, in_features)");
  TORCH_CHECK_VALUE(block_size > 0 && x.size(1) % block_size == 0 && out_features % block_size == 0,
                    "bcfft::forward: features (", x.size(1), ", ", out_features, ") not multiples of ", block_size);
  return at::empty({x.size(0), out_features}, x.options().dtype(out_dtype(x, bias)));
}

at::Tensor forward_glu_hip(const at::Tensor& x, const at::Tensor& spec_gu, int64_t block_size, int64_t gate_features,
                           int64_t algo) {
  require_device(x, "bcfft.forward_glu");
  TORCH_CHECK_VALUE(x.dim() == 2, "bcfft.forward_glu: x2d must be (N, in_features)");
  const int64_t n = x.size(0), k = x.size(1);
  if (block_size > 0 && gate_features % block_size == 0 && k % block_size == 0)
    check_spectra(spec_gu, 32 * ((gate_features / block_size + 15) / 16), k / block_size, block_size,
                  "bcfft.forward_glu");
  check_operand(spec_gu, x, "bcfft.forward_glu", "spectra", true);
  const c10::DeviceGuard guard(x.device());
  const at::Tensor xa = aligned(x);
  at::Tensor h = at::empty({n, gate_features}, x.options());
  if (n == 0) return h;
  const hipStream_t s = c10::hip::getCurrentHIPStream(x.device().index()).stream();
  check_status(bcfft_forward_glu_algo(xa.data_ptr(), dtype_code(xa.scalar_type()), n, (int)k, (int)gate_features,
                                      (int)block_size, spec_gu.data_ptr(), h.data_ptr(), (int)algo, s),
               "bcfft_forward_glu");
  return h;
}

at::Tensor forward_glu_meta(const at::Tensor& x, const at::Tensor& spec_gu, int64_t block_size, int64_t gate_features,
                            int64_t algo) {
  TORCH_CHECK_VALUE(x.dim() == 2 && block_size > 0 && x.size(1) % block_size == 0 && gate_features % block_size == 0,
                    "bcfft::forward_glu: x2d must be (N, in_features), features multiples of block_size");
  return at::empty({x.size(0), gate_features}, x.options());
}

// host tensors: the same loud error as the Python path (no CPU engine in the product)
at::Tensor forward_cpu(const at::Tensor& x, const at::Tensor&, const std::optional<at::Tensor>&, int64_t, int64_t,
                       int64_t, bool) {
  require_device(x, "bcfft.forward");
  return x;
}

at::Tensor forward_glu_cpu(const at::Tensor& x, const at::Tensor&, int64_t, int64_t, int64_t) {
  require_device(x, "bcfft.forward_glu");
  return x;
}

// Autograd key: these operators are forward-only (the module's backward is bcfft.ops' custom
// autograd Function over the same kernels, patch_llama_fft._BCFunction). Called directly with an
// input that requires grad under grad mode, they refuse instead of returning a tensor without a
// grad_fn (which would only warn at backward time); otherwise they dispatch below autograd.
bool wants_grad(const at::Tensor& t) { return t.defined() && t.requires_grad(); }

at::Tensor forward_autograd(const at::Tensor& x, const at::Tensor& spec, const std::optional<at::Tensor>& bias,
                            int64_t block_size, int64_t out_features, int64_t algo, bool split_k) {
  TORCH_CHECK(!(at::GradMode::is_enabled() && (wants_grad(x) || wants_grad(spec) || (bias && wants_grad(*bias)))),
              "torch.ops.bcfft_native.forward is forward-only: call it under torch.no_grad() / inference_mode, "
              "or use BlockCirculantLinear / bcfft.ops.forward, whose autograd Function has the backward");
  at::AutoDispatchBelowADInplaceOrView guard;
  static auto op = c10::Dispatcher::singleton()
                       .findSchemaOrThrow("bcfft_native::forward", "")
                       .typed<at::Tensor(const at::Tensor&, const at::Tensor&, const std::optional<at::Tensor>&,
                                         int64_t, int64_t, int64_t, bool)>();
  return op.call(x, spec, bias, block_size, out_features, algo, split_k);
}

at::Tensor forward_glu_autograd(const at::Tensor& x, const at::Tensor& spec_gu, int64_t block_size,
                                int64_t gate_features, int64_t algo) {
  TORCH_CHECK(!(at::GradMode::is_enabled() && (wants_grad(x) || wants_grad(spec_gu))),
              "torch.ops.bcfft_native.forward_glu is forward-only: call it under torch.no_grad() / "
              "inference_mode (the fused gate/up serves inference)");
  at::AutoDispatchBelowADInplaceOrView guard;
  static auto op = c10::Dispatcher::singleton()
                       .findSchemaOrThrow("bcfft_native::forward_glu", "")
                       .typed<at::Tensor(const at::Tensor&, const at::Tensor&, int64_t, int64_t, int64_t)>();
  return op.call(x, spec_gu, block_size, gate_features, algo);
}

}  // namespace

TORCH_LIBRARY(bcfft_native, m) {
  m.def("forward(Tensor x, Tensor spec, Tensor? bias, int block_size, int out_features, int algo, "
        "bool split_k=True) -> Tensor");
  m.def("forward_glu(Tensor x, Tensor spec_gu, int block_size, int gate_features, int algo) -> Tensor");
}

TORCH_LIBRARY_IMPL(bcfft_native, CUDA, m) {
  m.impl("forward", &forward_hip);
  m.impl("forward_glu", &forward_glu_hip);
}

TORCH_LIBRARY_IMPL(bcfft_native, Meta, m) {
  m.impl("forward", &forward_meta);
  m.impl("forward_glu", &forward_glu_meta);
}

TORCH_LIBRARY_IMPL(bcfft_native, CPU, m) {
  m.impl("forward", &forward_cpu);
  m.impl("forward_glu", &forward_glu_cpu);
}

TORCH_LIBRARY_IMPL(bcfft_native, Autograd, m) {
  m.impl("forward", &forward_autograd);
  m.impl("forward_glu", &forward_glu_autograd);
}
