// PyTorch / pybind11 bindings of the hipdsml native library (module `_C`).
//
// Tensor-facing entry points validate device, dtype, contiguity and sizes
// before any kernel is launched (a shape mismatch must never reach a kernel
// that assumes it).
#include <ATen/hip/HIPContext.h>
#include <pybind11/stl.h>
#include <torch/extension.h>

#include <rocprofiler-sdk-roctx/roctx.h>

#include "runtime/runtime.h"

namespace py = pybind11;
using namespace dsml;

namespace {

void check_cuda(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

void check_cuda_strided(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
}

void check_f32(const torch::Tensor& t, const char* name) {
  check_cuda(t, name);
  TORCH_CHECK(t.scalar_type() == torch::kFloat32, name, " must be float32");
}

int32_t dtype_of(const torch::Tensor& t) {
  switch (t.scalar_type()) {
    case torch::kFloat32: return kF32;
    case torch::kBFloat16: return kBF16;
    case torch::kFloat16: return kF16;
    case torch::kUInt8: return kU8;
    case torch::kInt32: return kI32;
    default: TORCH_CHECK(false, "unsupported dtype ", t.scalar_type());
  }
  return -1;
}

hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

void hip_ok(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, what, ": ", hipGetErrorString(e));
}

// Flat descriptor list, order fixed by models/mlp.py::MlpLayout.desc_list().
MlpDesc desc_from_list(const std::vector<int64_t>& v) {
  constexpr size_t kA = kMaxLayers + 1;
  const size_t want = 4 + 6 * kA + 1 + 2 * kMaxLayers + 2 * kA + 1;
  TORCH_CHECK(v.size() == want, "MlpDesc list has ", v.size(), " entries, expected ", want);
  MlpDesc d{};
  size_t p = 0;
  d.nlayers = (int32_t)v[p++];
  d.batch = (int32_t)v[p++];
  d.nbatches = (int32_t)v[p++];
  d.w_in_lds = (int32_t)v[p++];
  for (size_t i = 0; i < kA; ++i) d.dims[i] = (int32_t)v[p++];
  for (size_t i = 0; i < kA; ++i) d.lds_act[i] = (int32_t)v[p++];
  for (size_t i = 0; i < kA; ++i) d.lds_dz[i] = (int32_t)v[p++];
  for (size_t i = 0; i < kA; ++i) d.lds_stride[i] = (int32_t)v[p++];
  for (size_t i = 0; i < kA; ++i) d.lds_w[i] = (int32_t)v[p++];
  for (size_t i = 0; i < kA; ++i) d.lds_b[i] = (int32_t)v[p++];
  d.lds_floats = (int32_t)v[p++];
  for (int i = 0; i < kMaxLayers; ++i) d.w_off[i] = v[p++];
  for (int i = 0; i < kMaxLayers; ++i) d.b_off[i] = v[p++];
  for (size_t i = 0; i < kA; ++i) d.act_off[i] = v[p++];
  for (size_t i = 0; i < kA; ++i) d.dz_off[i] = v[p++];
  d.lab_off = v[p++];
  TORCH_CHECK(d.nlayers >= 1 && d.nlayers <= kMaxLayers, "nlayers out of range");
  TORCH_CHECK(d.batch >= 1 && d.nbatches >= 1, "batch / nbatches must be >= 1");
  for (int l = 0; l < d.nlayers; ++l) {
    TORCH_CHECK(d.dims[l] >= 4 && d.dims[l] % 4 == 0,
                "layer input dims must be multiples of 4 (dim ", l, " = ", d.dims[l], ")");
    TORCH_CHECK(d.w_off[l] % 4 == 0 && d.b_off[l] % 4 == 0, "param segments must be 16 B aligned");
  }
  TORCH_CHECK(d.dims[d.nlayers] >= 1, "output dim must be >= 1");
  return d;
}

int64_t layout_param_end(const MlpDesc& d) {
  int64_t end = 0;
  for (int l = 0; l < d.nlayers; ++l) {
    end = std::max<int64_t>(end, d.w_off[l] + (int64_t)d.dims[l + 1] * d.dims[l]);
    end = std::max<int64_t>(end, d.b_off[l] + d.dims[l + 1]);
  }
  return end;
}

int64_t layout_ws_end(const MlpDesc& d) {
  int64_t end = 0;
  for (int l = 1; l <= d.nlayers; ++l) {
    end = std::max<int64_t>(end, d.dz_off[l] + (int64_t)d.batch * d.dims[l]);
    if (l < d.nlayers) end = std::max<int64_t>(end, d.act_off[l] + (int64_t)d.batch * d.dims[l]);
  }
  return std::max<int64_t>(end, d.lab_off + d.batch);
}

struct PyMlpRunner {
  MlpDesc d;
  std::vector<torch::Tensor> keep;  // keep tensors alive while the runner exists
  // persistent-step operands: one slot each, replaced (not appended) on every
  // set_* call, so a released table is really freed
  torch::Tensor keep_xbuf, keep_err, keep_gram, keep_xall, keep_xact_in;
  std::unique_ptr<MlpRunner> r;
  hipStream_t stream = nullptr;
  bool own_stream = true;
  bool follow = false;  // run on torch's current stream at each call
  int device = 0;

  // stream_handle != 0: run on that (caller-owned) stream instead of a fresh
  // one.  Replicas of one process that spin on each other (the xGMI exchanges)
  // need streams on distinct hardware queues; HIP deals streams round-robin over
  // GPU_MAX_HW_QUEUES, so such groups take streams from a pool created back to
  // back once per process (parallel/xchg.py replica_streams) rather than
  // whatever queue a stream created later in a long process lands on.
  // follow_torch: every call runs on torch's CURRENT stream (PyTorch's own
  // convention), so work the caller enqueued before is ordered ahead of the
  // steps by the stream itself -- no cross-queue event edge per call.  The
  // runner's own stream is then used only to capture graphs.
  PyMlpRunner(const std::vector<int64_t>& desc, torch::Tensor X, torch::Tensor labels,
              torch::Tensor P, torch::Tensor G, torch::Tensor V, torch::Tensor ws,
              torch::Tensor slab, torch::Tensor ctr, torch::Tensor stats, float lr, float momentum,
              float weight_decay, uintptr_t stream_handle, bool follow_torch) {
    d = desc_from_list(desc);
    check_f32(X, "X");
    check_f32(P, "params");
    check_f32(G, "grads");
    check_f32(ws, "workspace");
    check_f32(slab, "slab");
    check_f32(stats, "stats");
    check_cuda(labels, "labels");
    check_cuda(ctr, "ctr");
    TORCH_CHECK(labels.scalar_type() == torch::kInt32, "labels must be int32");
    TORCH_CHECK(ctr.scalar_type() == torch::kInt64 && ctr.numel() >= 2, "ctr must be int64[2]");
    TORCH_CHECK(stats.numel() >= 3, "stats must hold 3 floats");
    TORCH_CHECK(X.dim() == 2 && X.size(1) >= d.dims[0] && X.size(1) % 4 == 0,
                "X must be [nsamples, >=d0] with a row stride multiple of 4");
    TORCH_CHECK(X.size(0) >= (int64_t)d.batch * d.nbatches, "X has fewer rows than batch*nbatches");
    TORCH_CHECK(labels.numel() >= (int64_t)d.batch * d.nbatches, "labels too short");
    TORCH_CHECK(P.numel() >= layout_param_end(d) && G.numel() == P.numel(),
                "params/grads too small for the layout");
    TORCH_CHECK(ws.numel() >= layout_ws_end(d), "workspace too small for the layout");
    const MlpLaunchCfg c = mlp_plan_first_layer(d);
    TORCH_CHECK(slab.numel() >= (int64_t)c.nsplit * d.batch * d.dims[1], "slab too small (need ",
                (int64_t)c.nsplit * d.batch * d.dims[1], ")");
    const bool need_v = momentum != 0.f || weight_decay != 0.f;
    if (need_v) {
      check_f32(V, "velocity");
      TORCH_CHECK(V.numel() == P.numel(), "velocity must match params");
    }
    device = X.get_device();
    keep = {X, labels, P, G, V, ws, slab, ctr, stats};
    MlpBuffers b;
    b.X = X.data_ptr<float>();
    b.ldx = X.size(1);
    b.labels = labels.data_ptr<int32_t>();
    b.P = P.data_ptr<float>();
    b.G = G.data_ptr<float>();
    b.V = need_v ? V.data_ptr<float>() : nullptr;
    b.ws = ws.data_ptr<float>();
    b.slab = slab.data_ptr<float>();
    b.ctr = ctr.data_ptr<int64_t>();
    b.stats = stats.data_ptr<float>();
    b.nparams = P.numel();
    hip_ok(hipSetDevice(device), "hipSetDevice");
    if (stream_handle != 0) {
      stream = reinterpret_cast<hipStream_t>(stream_handle);
      own_stream = false;
    } else {
      hip_ok(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking), "hipStreamCreate");
      follow = follow_torch;
    }
    r = std::make_unique<MlpRunner>(d, b, lr, momentum, weight_decay);
  }
  ~PyMlpRunner() {
    if (follow) (void)hipStreamSynchronize(cur_stream());
    r.reset();
    if (stream) (void)hipStreamSynchronize(stream);
    if (ev_in) (void)hipEventDestroy(ev_in);
    if (ev_out) (void)hipEventDestroy(ev_out);
    if (stream && own_stream) (void)hipStreamDestroy(stream);
  }
  // All runner work goes on the runner's own stream; join with torch's stream
  // first so tensors initialised by torch are visible.
  // Reused events for the two stream edges (no create/destroy per call).
  hipEvent_t ev_in = nullptr, ev_out = nullptr;
  hipEvent_t edge_event(hipEvent_t& e) {
    if (e == nullptr)
      hip_ok(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    return e;
  }
  hipStream_t run_stream() const { return follow ? cur_stream() : stream; }
  void join_torch() {
    if (follow) return;
    hipEvent_t e = edge_event(ev_in);
    hip_ok(hipEventRecord(e, cur_stream()), "hipEventRecord");
    hip_ok(hipStreamWaitEvent(stream, e, 0), "hipStreamWaitEvent");
  }
  // The reverse edge: torch's current stream waits for everything enqueued on
  // the runner's stream.  A host-side synchronize alone is not enough for a
  // consumer on another queue: with per-XCD L2s it can still read lines it
  // cached before the runner's kernels wrote them back (tests/test_gpu_xchg.py).
  void join_into_torch() {
    if (follow) return;
    hipEvent_t e = edge_event(ev_out);
    hip_ok(hipEventRecord(e, stream), "hipEventRecord");
    hip_ok(hipStreamWaitEvent(cur_stream(), e, 0), "hipStreamWaitEvent");
  }
  // join = false: the caller knows torch enqueued nothing the steps read since
  // the last join (saves the cross-queue barrier packet).
  void step(int n, bool join) {
    if (join) join_torch();
    r->enqueue_steps(n, run_stream());
  }
  void fwd_bwd() { join_torch(); r->enqueue_fwd_bwd(run_stream()); }
  void update() { join_torch(); r->enqueue_update(run_stream()); }
  // Graphs are captured on the runner's own stream (never the legacy null
  // stream) after it has caught up with torch's current stream.
  void capture(int steps, bool capture_comm) {
    hipEvent_t e = edge_event(ev_in);
    hip_ok(hipEventRecord(e, cur_stream()), "hipEventRecord");
    hip_ok(hipStreamWaitEvent(stream, e, 0), "hipStreamWaitEvent");
    hip_ok(hipStreamSynchronize(stream), "sync");
    r->capture(steps, capture_comm, stream);
  }
  void replay(int times, int steps) {
    hipStream_t s = run_stream();
    for (int i = 0; i < times; ++i) r->replay(s, steps);
  }
  void synchronize() {
    hipStream_t s = run_stream();
    py::gil_scoped_release nogil;
    hip_ok(hipStreamSynchronize(s), "hipStreamSynchronize");
  }
  uintptr_t stream_handle() const { return reinterpret_cast<uintptr_t>(run_stream()); }
};

struct PyComm {
  std::unique_ptr<RcclComm> c;
  PyComm(py::bytes uid, int rank, int nranks, int device, bool blocking) {
    std::string s = uid;
    std::vector<uint8_t> v(s.begin(), s.end());
    py::gil_scoped_release nogil;  // init is collective: do not hold the GIL
    c = std::make_unique<RcclComm>(v, rank, nranks, device, blocking);
  }
};

RcclComm* live(PyComm& s) {
  if (!s.c) throw std::runtime_error("RcclComm used after destroy()");
  return s.c.get();
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "hipdsml native MI355X (gfx950) kernels and device runtime";

  // ---- elementwise --------------------------------------------------------
  m.def("sgd_update_", [](torch::Tensor P, torch::Tensor G, double scale) {
    check_f32(P, "P"); check_f32(G, "G");
    TORCH_CHECK(P.numel() == G.numel(), "P/G size mismatch");
    hip_ok(sgd_update_f32(P.data_ptr<float>(), G.data_ptr<float>(), P.numel(), (float)scale,
                          cur_stream()), "sgd_update_f32");
  });
  m.def("sgd_momentum_", [](torch::Tensor P, torch::Tensor G, torch::Tensor V, double lr,
                            double mom, double wd, double gscale) {
    check_f32(P, "P"); check_f32(G, "G"); check_f32(V, "V");
    TORCH_CHECK(P.numel() == G.numel() && P.numel() == V.numel(), "P/G/V size mismatch");
    hip_ok(sgd_momentum_f32(P.data_ptr<float>(), G.data_ptr<float>(), V.data_ptr<float>(),
                            P.numel(), (float)lr, (float)mom, (float)wd, (float)gscale,
                            cur_stream()), "sgd_momentum_f32");
  });
  m.def("reduce_into", [](torch::Tensor dst, torch::Tensor a, torch::Tensor b, int op) {
    check_cuda(dst, "dst"); check_cuda(a, "a"); check_cuda(b, "b");
    TORCH_CHECK(dst.scalar_type() == a.scalar_type() && a.scalar_type() == b.scalar_type(),
                "dtype mismatch");
    TORCH_CHECK(dst.numel() == a.numel() && a.numel() == b.numel(), "size mismatch");
    hip_ok(reduce_into(dst.data_ptr(), a.data_ptr(), b.data_ptr(), dst.numel(), dtype_of(dst), op,
                       cur_stream()), "reduce_into");
  });
  m.def("reduce_multi_", [](const std::vector<torch::Tensor>& dsts, const std::vector<torch::Tensor>& srcs,
                             int op) {
    TORCH_CHECK(dsts.size() == srcs.size() && !dsts.empty() && dsts.size() <= (size_t)kMaxReduceSegs,
                "reduce_multi_: 1..", kMaxReduceSegs, " (dst, src) pairs");
    ReduceSegs m{};
    const int32_t dt = dtype_of(dsts[0]);
    for (size_t k = 0; k < dsts.size(); ++k) {
      TORCH_CHECK(dsts[k].is_cuda() && srcs[k].is_cuda() && dsts[k].is_contiguous() &&
                  srcs[k].is_contiguous() && dsts[k].numel() == srcs[k].numel() &&
                  dtype_of(dsts[k]) == dt && dtype_of(srcs[k]) == dt, "reduce_multi_: pair ", k);
      m.seg[m.count++] = ReduceSeg{dsts[k].data_ptr(), srcs[k].data_ptr(), dsts[k].numel()};
    }
    hip_ok(reduce_multi_inplace(m, dt, op, cur_stream()), "reduce_multi_inplace");
  });
  m.def("scale_", [](torch::Tensor x, double alpha) {
    check_cuda(x, "x");
    hip_ok(scale_inplace(x.data_ptr(), x.numel(), dtype_of(x), (float)alpha, cur_stream()),
           "scale_inplace");
  });
  m.def("u8_to_f32", [](torch::Tensor dst, torch::Tensor src, double scale) {
    check_f32(dst, "dst"); check_cuda(src, "src");
    TORCH_CHECK(src.scalar_type() == torch::kUInt8 && src.numel() == dst.numel(), "bad src");
    hip_ok(u8_to_f32_scaled(dst.data_ptr<float>(), src.data_ptr<uint8_t>(), dst.numel(),
                            (float)scale, cur_stream()), "u8_to_f32");
  });
  m.def("f32_to_bf16", [](torch::Tensor dst, torch::Tensor src) {
    check_f32(src, "src"); check_cuda(dst, "dst");
    TORCH_CHECK(dst.scalar_type() == torch::kBFloat16 && dst.numel() == src.numel(), "bad dst");
    hip_ok(f32_to_bf16(reinterpret_cast<uint16_t*>(dst.data_ptr()), src.data_ptr<float>(),
                       src.numel(), cur_stream()), "f32_to_bf16");
  });
  m.def("bf16_to_f32", [](torch::Tensor dst, torch::Tensor src) {
    check_f32(dst, "dst"); check_cuda(src, "src");
    TORCH_CHECK(src.scalar_type() == torch::kBFloat16 && dst.numel() == src.numel(), "bad src");
    hip_ok(bf16_to_f32(dst.data_ptr<float>(), reinterpret_cast<const uint16_t*>(src.data_ptr()),
                       src.numel(), cur_stream()), "bf16_to_f32");
  });

  // ---- bf16 GEMM toolkit (wide MLP) -------------------------------------------
  auto bf16p = [](const torch::Tensor& t, const char* name) -> uint16_t* {
    check_cuda_strided(t, name);
    TORCH_CHECK(t.scalar_type() == torch::kBFloat16, name, " must be bfloat16");
    return reinterpret_cast<uint16_t*>(t.data_ptr());
  };
  m.def("gemm_bf16_nt", [bf16p](torch::Tensor A, torch::Tensor B, torch::Tensor Cp, int64_t M,
                               int64_t N, int64_t K, int64_t splits) {
    TORCH_CHECK(A.dim() == 2 && B.dim() == 2, "A, B must be 2-D");
    TORCH_CHECK(A.stride(1) == 1 && B.stride(1) == 1, "A, B rows must be contiguous");
    TORCH_CHECK(A.size(0) >= M && B.size(0) >= N && A.size(1) >= K && B.size(1) >= K, "A/B too small");
    check_f32(Cp, "Cp");
    const int S = gemm_bf16_num_splits((int)K, (int)splits);
    TORCH_CHECK(Cp.numel() >= (int64_t)S * M * N, "Cp too small: need ", (int64_t)S * M * N);
    hip_ok(gemm_bf16_nt(bf16p(A, "A"), A.stride(0), bf16p(B, "B"), B.stride(0), Cp.data_ptr<float>(),
                        (int)M, (int)N, (int)K, (int)splits, cur_stream()), "gemm_bf16_nt");
    return S;
  });
  m.def("gemm_num_splits", [](int64_t K, int64_t splits) { return gemm_bf16_num_splits((int)K, (int)splits); });
  m.def("gemm_epilogue", [bf16p](torch::Tensor Cp, int64_t S, int64_t M, int64_t N, double alpha,
                                c10::optional<torch::Tensor> bias, bool relu,
                                c10::optional<torch::Tensor> mask, c10::optional<torch::Tensor> of32,
                                c10::optional<torch::Tensor> obf, c10::optional<torch::Tensor> obfT) {
    check_f32(Cp, "Cp");
    TORCH_CHECK(Cp.numel() >= S * M * N, "Cp too small");
    const float* b = nullptr;
    if (bias) { check_f32(*bias, "bias"); TORCH_CHECK(bias->numel() >= N, "bias too small"); b = bias->data_ptr<float>(); }
    auto chk2 = [&](const torch::Tensor& t, int64_t r, int64_t c, const char* nm) {
      TORCH_CHECK(t.dim() == 2 && t.stride(1) == 1 && t.size(0) >= r && t.size(1) >= c, nm, " shape");
    };
    const uint16_t* mk = nullptr; int64_t ldm = 0;
    if (mask) { chk2(*mask, M, N, "mask"); mk = bf16p(*mask, "mask"); ldm = mask->stride(0); }
    float* o32 = nullptr; int64_t ldo = 0;
    if (of32) { check_cuda_strided(*of32, "of32"); TORCH_CHECK(of32->scalar_type() == torch::kFloat32, "of32 f32");
                chk2(*of32, M, N, "of32"); o32 = of32->data_ptr<float>(); ldo = of32->stride(0); }
    uint16_t* ob = nullptr; int64_t ldb = 0;
    if (obf) { chk2(*obf, M, N, "obf"); ob = bf16p(*obf, "obf"); ldb = obf->stride(0); }
    uint16_t* obt = nullptr; int64_t ldt = 0;
    if (obfT) { chk2(*obfT, N, M, "obfT"); obt = bf16p(*obfT, "obfT"); ldt = obfT->stride(0); }
    hip_ok(gemm_epilogue(Cp.data_ptr<float>(), (int)S, (int)M, (int)N, (float)alpha, b, relu ? 1 : 0,
                         mk, ldm, o32, ldo, ob, ldb, obt, ldt, cur_stream()), "gemm_epilogue");
  }, py::arg("Cp"), py::arg("S"), py::arg("M"), py::arg("N"), py::arg("alpha") = 1.0,
     py::arg("bias") = py::none(), py::arg("relu") = false, py::arg("mask") = py::none(),
     py::arg("of32") = py::none(), py::arg("obf") = py::none(), py::arg("obfT") = py::none());
  m.def("cast_transpose", [bf16p](torch::Tensor X, int64_t M, int64_t K, torch::Tensor Y,
                                 c10::optional<torch::Tensor> YT) {
    check_f32(X, "X");
    TORCH_CHECK(X.dim() == 2 && X.size(0) >= M && X.size(1) >= K, "X shape");
    TORCH_CHECK(Y.dim() == 2 && Y.size(0) >= M && Y.stride(1) == 1, "Y shape");
    const int64_t Kp = Y.size(1);
    TORCH_CHECK(Kp >= K, "Y narrower than K");
    uint16_t* yt = nullptr; int64_t ldt = 0;
    if (YT) { TORCH_CHECK(YT->dim() == 2 && YT->size(0) >= Kp && YT->size(1) >= M && YT->stride(1) == 1, "YT shape");
              yt = bf16p(*YT, "YT"); ldt = YT->stride(0); }
    hip_ok(cast_transpose(X.data_ptr<float>(), X.stride(0), (int)M, (int)K, (int)Kp, bf16p(Y, "Y"),
                          Y.stride(0), yt, ldt, cur_stream()), "cast_transpose");
  });
  m.def("softmax_xent", [bf16p](torch::Tensor logits, torch::Tensor labels, int64_t B, int64_t C,
                               double inv_batch, torch::Tensor dz, c10::optional<torch::Tensor> dzT,
                               torch::Tensor stats) {
    check_f32(logits, "logits"); check_cuda(labels, "labels"); check_f32(stats, "stats");
    TORCH_CHECK(labels.scalar_type() == torch::kInt32 && labels.numel() >= B, "labels");
    TORCH_CHECK(logits.dim() == 2 && logits.size(0) >= B && logits.size(1) >= C, "logits shape");
    TORCH_CHECK(dz.dim() == 2 && dz.size(0) >= B && dz.stride(1) == 1, "dz shape");
    const int64_t Cp = dz.size(1);
    uint16_t* t = nullptr; int64_t ldt = 0;
    if (dzT) { TORCH_CHECK(dzT->dim() == 2 && dzT->size(0) >= Cp && dzT->size(1) >= B, "dzT shape");
               t = bf16p(*dzT, "dzT"); ldt = dzT->stride(0); }
    hip_ok(softmax_xent(logits.data_ptr<float>(), logits.stride(0), labels.data_ptr<int32_t>(), (int)B,
                        (int)C, (int)Cp, (float)inv_batch, bf16p(dz, "dz"), dz.stride(0), t, ldt,
                        stats.data_ptr<float>(), cur_stream()), "softmax_xent");
  });
  m.def("head_softmax_xent", [bf16p](torch::Tensor H, torch::Tensor W, c10::optional<torch::Tensor> bias,
                                    int64_t B, int64_t K, int64_t C, torch::Tensor labels,
                                    double inv_batch, c10::optional<torch::Tensor> logits,
                                    torch::Tensor dz, c10::optional<torch::Tensor> dzT,
                                    torch::Tensor stats, c10::optional<torch::Tensor> dzp,
                                    c10::optional<torch::Tensor> dzpT, bool row_stats,
                                    c10::optional<torch::Tensor> hs, int64_t hs_splits,
                                    c10::optional<torch::Tensor> hs_bias, bool hs_relu, double hs_alpha) {
    TORCH_CHECK(!row_stats || stats.numel() >= 4 * B, "row_stats needs 4 floats per row");
    TORCH_CHECK(H.dim() == 2 && H.stride(1) == 1 && H.size(0) >= B && H.size(1) >= K, "H shape");
    TORCH_CHECK(W.dim() == 2 && W.stride(1) == 1 && W.size(0) >= C && W.size(1) >= K, "W shape");
    check_cuda(labels, "labels"); check_f32(stats, "stats");
    TORCH_CHECK(labels.scalar_type() == torch::kInt32 && labels.numel() >= B, "labels");
    const float* b = nullptr;
    if (bias) { check_f32(*bias, "bias"); TORCH_CHECK(bias->numel() >= C, "bias"); b = bias->data_ptr<float>(); }
    float* lg = nullptr; int64_t ldl = 0;
    if (logits) { check_f32(*logits, "logits"); TORCH_CHECK(logits->dim() == 2 && logits->size(0) >= B && logits->size(1) >= C, "logits shape");
                  lg = logits->data_ptr<float>(); ldl = logits->stride(0); }
    TORCH_CHECK(dz.dim() == 2 && dz.size(0) >= B && dz.stride(1) == 1, "dz shape");
    const int64_t Cp = dz.size(1);
    uint16_t* t = nullptr; int64_t ldt = 0;
    if (dzT) { TORCH_CHECK(dzT->dim() == 2 && dzT->size(0) >= Cp && dzT->size(1) >= B, "dzT shape");
               t = bf16p(*dzT, "dzT"); ldt = dzT->stride(0); }
    uint16_t* pp = nullptr; int64_t ldp = 0; uint16_t* ppT = nullptr; int64_t ldpT = 0;
    if (dzp) { TORCH_CHECK(dzp->dim() == 2 && dzp->stride(1) == 1 && dzp->size(0) >= B && dzp->size(1) >= K, "dzp shape");
               pp = bf16p(*dzp, "dzp"); ldp = dzp->stride(0); }
    if (dzpT) { TORCH_CHECK(dzp && dzpT->dim() == 2 && dzpT->stride(1) == 1 && dzpT->size(0) >= K && dzpT->size(1) >= B,
                            "dzpT shape (needs dzp)");
                ppT = bf16p(*dzpT, "dzpT"); ldpT = dzpT->stride(0); }
    HeadSlabs hsl{};
    if (hs) {
      // H is OUTPUT here: the raw split-K slices of the last hidden layer's GEMM
      // (gemm_skinny raw=True), combined + epilogue on load, H written back
      check_f32(*hs, "hs");
      const int64_t stride = hs->numel() / std::max<int64_t>(1, hs_splits);
      TORCH_CHECK(hs_splits >= 1 && stride >= (K / 64) * 4096, "hs: hs_splits slices of K/64 tiles x 4096");
      hsl.slabs = hs->data_ptr<float>();
      hsl.S = (int)hs_splits;
      hsl.stride = (K / 64) * 4096;
      hsl.alpha = (float)hs_alpha;
      if (hs_bias) { check_f32(*hs_bias, "hs_bias"); TORCH_CHECK(hs_bias->numel() >= K, "hs_bias");
                     hsl.bias = hs_bias->data_ptr<float>(); }
      hsl.relu = hs_relu ? 1 : 0;
      hsl.Hout = bf16p(H, "H");
      hsl.ldo = H.stride(0);
    }
    hip_ok(head_softmax_xent(bf16p(H, "H"), H.stride(0), bf16p(W, "W"), W.stride(0), b, (int)B, (int)K,
                             (int)C, labels.data_ptr<int32_t>(), (float)inv_batch, lg, ldl,
                             bf16p(dz, "dz"), dz.stride(0), t, ldt, (int)Cp, stats.data_ptr<float>(),
                             cur_stream(), pp, ldp, ppT, ldpT, row_stats ? 1 : 0, hs ? &hsl : nullptr),
           "head_softmax_xent");
  }, py::arg("H"), py::arg("W"), py::arg("bias"), py::arg("B"), py::arg("K"), py::arg("C"),
     py::arg("labels"), py::arg("inv_batch"), py::arg("logits"), py::arg("dz"), py::arg("dzT"),
     py::arg("stats"), py::arg("dzp") = py::none(), py::arg("dzpT") = py::none(),
     py::arg("row_stats") = false, py::arg("hs") = py::none(), py::arg("hs_splits") = 0,
     py::arg("hs_bias") = py::none(), py::arg("hs_relu") = true, py::arg("hs_alpha") = 1.0);
  m.def("rowsum_bf16", [bf16p](torch::Tensor X, int64_t N, int64_t cols, c10::optional<torch::Tensor> out,
                              c10::optional<torch::Tensor> bias, double lr) {
    TORCH_CHECK(X.dim() == 2 && X.size(0) >= N && X.size(1) >= cols, "X shape");
    TORCH_CHECK(out.has_value() != bias.has_value(), "exactly one of out / bias");
    torch::Tensor t = out ? *out : *bias;
    check_f32(t, "out/bias");
    TORCH_CHECK(t.numel() >= N, "out/bias too small");
    hip_ok(rowsum_bf16(bf16p(X, "X"), X.stride(0), (int)N, (int)cols, out ? t.data_ptr<float>() : nullptr,
                       bias ? t.data_ptr<float>() : nullptr, (float)lr, cur_stream()), "rowsum_bf16");
  }, py::arg("X"), py::arg("N"), py::arg("cols"), py::arg("out") = py::none(), py::arg("bias") = py::none(),
     py::arg("lr") = 0.0);
  m.def("gemm_bf16_nt_fused", [bf16p](torch::Tensor A, torch::Tensor B, int64_t M, int64_t N, int64_t K,
                                     double alpha, c10::optional<torch::Tensor> bias, bool relu,
                                     c10::optional<torch::Tensor> mask, c10::optional<torch::Tensor> of32,
                                     c10::optional<torch::Tensor> obf, c10::optional<torch::Tensor> obfT,
                                     c10::optional<torch::Tensor> sgdW, double lr, int64_t splits,
                                     c10::optional<torch::Tensor> ws, c10::optional<torch::Tensor> ctr,
                                     c10::optional<torch::Tensor> bgrad,
                                     c10::optional<torch::Tensor> bsgd) {
    // A 3-D = k-blocked [K / 32 blocks][rows][32] (rows64 only): element (m, k) at
    // A[k / 32][m][k % 32]
    const bool ablk = A.dim() == 3;
    TORCH_CHECK(!ablk || (splits == 0 && A.stride(2) == 1 && A.stride(1) == 32 && A.size(2) == 32 &&
                          A.size(0) * 32 >= K && A.size(1) >= M), "k-blocked A: [>= K/32][>= M][32], splits=0");
    TORCH_CHECK((ablk || (A.dim() == 2 && A.stride(1) == 1)) && B.dim() == 2 && B.stride(1) == 1, "A, B 2-D rows");
    TORCH_CHECK((ablk || (A.size(0) >= M && A.size(1) >= K)) && B.size(0) >= N && B.size(1) >= K, "A/B too small");
    auto chk2 = [&](const torch::Tensor& t, int64_t r, int64_t c, const char* nm) {
      TORCH_CHECK(t.is_cuda() && t.dim() == 2 && t.stride(1) == 1 && t.size(0) >= r && t.size(1) >= c, nm, " shape");
    };
    GemmEpi e{};
    e.alpha = (float)alpha;
    e.relu = relu ? 1 : 0;
    e.lr = (float)lr;
    if (bias) { check_f32(*bias, "bias"); TORCH_CHECK(bias->numel() >= N, "bias"); e.bias = bias->data_ptr<float>(); }
    if (mask) { chk2(*mask, M, N, "mask"); e.mask = bf16p(*mask, "mask"); e.ldm = mask->stride(0); }
    if (of32) { chk2(*of32, M, N, "of32"); TORCH_CHECK(of32->scalar_type() == torch::kFloat32, "of32 f32");
                e.of32 = of32->data_ptr<float>(); e.ldo = of32->stride(0); }
    if (obf) { chk2(*obf, M, N, "obf"); e.obf = bf16p(*obf, "obf"); e.ldb = obf->stride(0); }
    if (obfT) { chk2(*obfT, N, M, "obfT"); e.obfT = bf16p(*obfT, "obfT"); e.ldt = obfT->stride(0); }
    if (sgdW) { chk2(*sgdW, M, N, "sgdW"); TORCH_CHECK(sgdW->scalar_type() == torch::kFloat32, "sgdW f32");
                e.sgdW = sgdW->data_ptr<float>(); e.ldw = sgdW->stride(0); }
    if (bgrad) { check_f32(*bgrad, "bgrad"); TORCH_CHECK(bgrad->numel() >= M, "bgrad"); e.bgrad = bgrad->data_ptr<float>(); }
    if (bsgd) { check_f32(*bsgd, "bsgd"); TORCH_CHECK(bsgd->numel() >= M, "bsgd"); e.bsgd = bsgd->data_ptr<float>(); }
    if (splits == 0) {  // batch-row kernel: full K per block, epilogue fused, no slabs
      hip_ok(gemm_bf16_rows64(bf16p(A, "A"), A.stride(0), bf16p(B, "B"), B.stride(0), (int)M, (int)N,
                              (int)K, e, cur_stream(), ablk), "gemm_bf16_rows64");
      return 1;
    }
    const int S = gemm_bf16_num_splits((int)K, (int)splits);
    float* cp = nullptr;
    int* tc = nullptr;
    if (S > 1) {
      TORCH_CHECK(ws && ctr, "split-K fused GEMM needs ws (slabs) and ctr (tile counters)");
      check_f32(*ws, "ws");
      const int64_t tiles = ((N + 63) / 64) * ((M + 63) / 64);
      TORCH_CHECK(ws->numel() >= (int64_t)S * tiles * 4096, "ws too small: need ", (int64_t)S * tiles * 4096);
      check_cuda(*ctr, "ctr");
      TORCH_CHECK(ctr->scalar_type() == torch::kInt32 &&
                  ctr->numel() >= ((N + 63) / 64) * ((M + 63) / 64), "ctr: int32, one per 64x64 tile");
      cp = ws->data_ptr<float>();
      tc = ctr->data_ptr<int32_t>();
    }
    hip_ok(gemm_bf16_nt(bf16p(A, "A"), A.stride(0), bf16p(B, "B"), B.stride(0), cp, (int)M, (int)N,
                        (int)K, (int)splits, cur_stream(), &e, tc), "gemm_bf16_nt_fused");
    return S;
  }, py::arg("A"), py::arg("B"), py::arg("M"), py::arg("N"), py::arg("K"), py::arg("alpha") = 1.0,
     py::arg("bias") = py::none(), py::arg("relu") = false, py::arg("mask") = py::none(),
     py::arg("of32") = py::none(), py::arg("obf") = py::none(), py::arg("obfT") = py::none(),
     py::arg("sgdW") = py::none(), py::arg("lr") = 0.0, py::arg("splits") = 1,
     py::arg("ws") = py::none(), py::arg("ctr") = py::none(), py::arg("bgrad") = py::none(),
     py::arg("bsgd") = py::none());
  m.def("gemm_skinny_ws", [](int64_t M, int64_t N, int64_t K, int64_t splits) {
    int64_t wsw = 0, ctw = 0;
    gemm_skinny_ws((int)M, (int)N, (int)K, (int)splits, &wsw, &ctw);
    return py::make_tuple(wsw, ctw);
  }, py::arg("M"), py::arg("N"), py::arg("K"), py::arg("splits") = 0,
     "split-K workspace of a skinny GEMM: (fp32 words of ws, int32 words of ctr), both zeroed once");
  m.def("gemm_skinny", [bf16p](torch::Tensor A, torch::Tensor B, int64_t M, int64_t N, int64_t K, bool nn,
                              double alpha, c10::optional<torch::Tensor> bias, bool relu,
                              c10::optional<torch::Tensor> mask, c10::optional<torch::Tensor> of32,
                              c10::optional<torch::Tensor> obf, c10::optional<torch::Tensor> obfT,
                              int64_t splits, c10::optional<torch::Tensor> ws,
                              c10::optional<torch::Tensor> ctr, bool raw) {
    TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.stride(1) == 1 && B.stride(1) == 1, "A, B 2-D rows");
    TORCH_CHECK(A.size(0) >= M && A.size(1) >= K, "A too small");
    TORCH_CHECK(nn ? (B.size(0) >= K && B.size(1) >= N) : (B.size(0) >= N && B.size(1) >= K), "B too small");
    auto chk2 = [&](const torch::Tensor& t, int64_t r, int64_t c, const char* nm) {
      TORCH_CHECK(t.is_cuda() && t.dim() == 2 && t.stride(1) == 1 && t.size(0) >= r && t.size(1) >= c, nm, " shape");
    };
    GemmEpi e{};
    e.alpha = (float)alpha;
    e.relu = relu ? 1 : 0;
    if (bias) { check_f32(*bias, "bias"); TORCH_CHECK(bias->numel() >= N, "bias"); e.bias = bias->data_ptr<float>(); }
    if (mask) { chk2(*mask, M, N, "mask"); e.mask = bf16p(*mask, "mask"); e.ldm = mask->stride(0); }
    if (of32) { chk2(*of32, M, N, "of32"); TORCH_CHECK(of32->scalar_type() == torch::kFloat32, "of32 f32");
                e.of32 = of32->data_ptr<float>(); e.ldo = of32->stride(0); }
    if (obf) { chk2(*obf, M, N, "obf"); e.obf = bf16p(*obf, "obf"); e.ldb = obf->stride(0); }
    if (obfT) { chk2(*obfT, N, M, "obfT"); e.obfT = bf16p(*obfT, "obfT"); e.ldt = obfT->stride(0); }
    const int S = gemm_skinny_splits((int)M, (int)N, (int)K, (int)splits);
    float* cp = nullptr;
    int* tc = nullptr;
    if (raw) {
      // consumer-combined: every slice's partial tile into ws, no epilogue here
      TORCH_CHECK(ws && !bias && !mask && !of32 && !obf && !obfT,
                  "raw skinny GEMM: ws only (the consumer applies the epilogue)");
      check_f32(*ws, "ws");
      const int64_t tiles = ((N + 63) / 64) * ((M + 63) / 64);
      TORCH_CHECK(ws->numel() >= (int64_t)S * tiles * 4096, "ws too small for the raw slices");
      cp = ws->data_ptr<float>();
    } else if (S > 1) {
      TORCH_CHECK(ws && ctr, "split-K skinny GEMM needs ws (slabs) and ctr (tile counters)");
      check_f32(*ws, "ws");
      int64_t wsw = 0, ctw = 0;
      gemm_skinny_ws((int)M, (int)N, (int)K, (int)splits, &wsw, &ctw);
      TORCH_CHECK(ws->numel() >= wsw, "ws too small: need ", wsw);
      check_cuda(*ctr, "ctr");
      TORCH_CHECK(ctr->scalar_type() == torch::kInt32 && ctr->numel() >= ctw,
                  "ctr: int32, one per 64x64 tile: need ", ctw);
      cp = ws->data_ptr<float>();
      tc = ctr->data_ptr<int32_t>();
    }
    hip_ok(gemm_skinny(bf16p(A, "A"), A.stride(0), bf16p(B, "B"), B.stride(0), (int)M, (int)N, (int)K, nn,
                       (int)splits, cp, tc, e, cur_stream(), raw), "gemm_skinny");
    return S;
  }, py::arg("A"), py::arg("B"), py::arg("M"), py::arg("N"), py::arg("K"), py::arg("nn") = false,
     py::arg("alpha") = 1.0, py::arg("bias") = py::none(), py::arg("relu") = false,
     py::arg("mask") = py::none(), py::arg("of32") = py::none(), py::arg("obf") = py::none(),
     py::arg("obfT") = py::none(), py::arg("splits") = 0, py::arg("ws") = py::none(),
     py::arg("ctr") = py::none(), py::arg("raw") = false);
  m.def("wgrad_sgd", [bf16p](torch::Tensor Z, torch::Tensor X, int64_t M, int64_t N, int64_t K, double alpha,
                            double lr, c10::optional<torch::Tensor> W, c10::optional<torch::Tensor> Wb,
                            c10::optional<torch::Tensor> G, c10::optional<torch::Tensor> bias,
                            c10::optional<torch::Tensor> bgrad, c10::optional<torch::Tensor> Wh,
                            c10::optional<torch::Tensor> Wl) {
    TORCH_CHECK(Z.dim() == 2 && X.dim() == 2 && Z.stride(1) == 1 && X.stride(1) == 1, "Z, X 2-D rows");
    TORCH_CHECK(Z.size(0) >= M && X.size(0) >= M && Z.size(1) >= ((N + 7) / 8) * 8 &&
                X.size(1) >= ((K + 7) / 8) * 8, "Z / X too small (rows padded to 8 columns)");
    auto chk2 = [&](const torch::Tensor& t, int64_t r, int64_t c, const char* nm) {
      TORCH_CHECK(t.is_cuda() && t.dim() == 2 && t.stride(1) == 1 && t.size(0) >= r && t.size(1) >= c, nm, " shape");
    };
    float* w = nullptr; int64_t ldw = 0;
    uint16_t* wb = nullptr; int64_t ldwb = 0;
    float* g = nullptr; int64_t ldg = 0;
    if (W) { chk2(*W, N, K, "W"); TORCH_CHECK(W->scalar_type() == torch::kFloat32, "W f32"); w = W->data_ptr<float>(); ldw = W->stride(0); }
    if (Wb) { chk2(*Wb, N, K, "Wb"); wb = bf16p(*Wb, "Wb"); ldwb = Wb->stride(0); }
    if (G) { chk2(*G, N, K, "G"); TORCH_CHECK(G->scalar_type() == torch::kFloat32, "G f32"); g = G->data_ptr<float>(); ldg = G->stride(0); }
    float* b = nullptr; float* bg = nullptr;
    if (bias) { check_f32(*bias, "bias"); TORCH_CHECK(bias->numel() >= N, "bias"); b = bias->data_ptr<float>(); }
    if (bgrad) { check_f32(*bgrad, "bgrad"); TORCH_CHECK(bgrad->numel() >= N, "bgrad"); bg = bgrad->data_ptr<float>(); }
    WgLayer a{bf16p(Z, "Z"), Z.stride(0), bf16p(X, "X"), X.stride(0), (int)M, (int)N, (int)K, (float)alpha,
              (float)lr, w, ldw, wb, ldwb, g, ldg, b, bg};
    if (Wh) { chk2(*Wh, N, K, "Wh"); a.Wh = bf16p(*Wh, "Wh"); a.ldwh = Wh->stride(0); }
    if (Wl) {
      chk2(*Wl, N, K, "Wl");
      TORCH_CHECK(Wl->scalar_type() == torch::kInt16, "Wl must be int16");
      a.Wl = reinterpret_cast<uint16_t*>(Wl->data_ptr<int16_t>()); a.ldwl = Wl->stride(0);
    }
    hip_ok(wgrad_sgd_multi(&a, 1, cur_stream(), 64), "wgrad_sgd");
  }, py::arg("Z"), py::arg("X"), py::arg("M"), py::arg("N"), py::arg("K"), py::arg("alpha") = 1.0,
     py::arg("lr") = 0.0, py::arg("W") = py::none(), py::arg("Wb") = py::none(), py::arg("G") = py::none(),
     py::arg("bias") = py::none(), py::arg("bgrad") = py::none(), py::arg("Wh") = py::none(),
     py::arg("Wl") = py::none());
  m.def("hilo_sgd", [bf16p](torch::Tensor hic, torch::Tensor lo, c10::optional<torch::Tensor> G, double lr,
                           torch::Tensor hin) {
    // split master step: w = join(hic, lo) - lr * G; hin / lo <- split(w) (G [N x K] fp32)
    TORCH_CHECK(hic.dim() == 2 && lo.dim() == 2 && hin.dim() == 2 && hic.stride(1) == 1 && lo.stride(1) == 1 &&
                hin.stride(1) == 1, "hilo_sgd: 2-D rows");
    TORCH_CHECK(lo.scalar_type() == torch::kInt16, "lo must be int16");
    int64_t N = hic.size(0), K = hic.size(1);
    const float* g = nullptr; int64_t ldg = 0;
    if (G) {
      check_f32(*G, "G");
      TORCH_CHECK(G->dim() == 2 && G->stride(1) == 1, "G 2-D rows");
      N = G->size(0); K = G->size(1); g = G->data_ptr<float>(); ldg = G->stride(0);
    }
    TORCH_CHECK(hic.size(0) >= N && hic.size(1) >= K && lo.size(0) >= N && lo.size(1) >= K && hin.size(0) >= N &&
                hin.size(1) >= K, "hilo_sgd shapes");
    hip_ok(hilo_sgd(bf16p(hic, "hic"), hic.stride(0), reinterpret_cast<uint16_t*>(lo.data_ptr<int16_t>()),
                    lo.stride(0), g, ldg, (int)N, (int)K, (float)lr, bf16p(hin, "hin"), hin.stride(0), cur_stream()),
           "hilo_sgd");
  }, py::arg("hic"), py::arg("lo"), py::arg("G"), py::arg("lr"), py::arg("hin"));
  m.def("head_stamps", []() {
    std::vector<uint64_t> v(64 * 6);
    hip_ok(head_read_stamps(v.data()), "head_read_stamps");
    return v;
  });
  m.def("head_set_stamping", &head_set_stamping);
#ifdef HIPDSML_MEASURE
  m.def("head_set_debug", &head_set_debug);
  m.def("wide_input_stamps", []() {
    std::vector<uint64_t> v(1024 * 8);
    hip_ok(wide_input_read_stamps(v.data()), "wide_input_read_stamps");
    return v;
  });
  m.def("wide_input_set_stamping", &wide_input_set_stamping);
  m.def("wide_input_set_dbg", &wide_input_set_dbg);
  m.def("wgrad_rowblk_stamps", []() {
    std::vector<uint64_t> v(256 * 16);
    hip_ok(wgrad_rowblk_read_stamps(v.data()), "wgrad_rowblk_read_stamps");
    return v;
  });
  m.def("wgrad_rowblk_set_stamping", &wgrad_rowblk_set_stamping);
#endif
#ifdef HIPDSML_MEASURE
  m.attr("measure_build") = true;
#else
  m.attr("measure_build") = false;
#endif
  // one layer of the fused weight-gradient launches:
  // (Z, X, M, N, K, alpha, lr, W, Wb, G, bias, bgrad[, Wh, Wl]); tensors may be None
  auto wg_layer = [bf16p](py::handle it) -> WgLayer {
    auto opt = [](py::handle h) -> c10::optional<torch::Tensor> {
      if (h.is_none()) return c10::nullopt;
      return h.cast<torch::Tensor>();
    };
    py::tuple t = it.cast<py::tuple>();
    TORCH_CHECK(t.size() == 12 || t.size() == 14,
                "wgrad layer: (Z, X, M, N, K, alpha, lr, W, Wb, G, bias, bgrad[, Wh, Wl])");
    torch::Tensor Z = t[0].cast<torch::Tensor>(), X = t[1].cast<torch::Tensor>();
    const int64_t M = t[2].cast<int64_t>(), N = t[3].cast<int64_t>(), K = t[4].cast<int64_t>();
    TORCH_CHECK(Z.dim() == 2 && X.dim() == 2 && Z.stride(1) == 1 && X.stride(1) == 1, "Z, X 2-D rows");
    TORCH_CHECK(Z.size(0) >= M && X.size(0) >= M && Z.size(1) >= ((N + 7) / 8) * 8 &&
                X.size(1) >= ((K + 7) / 8) * 8, "Z / X too small");
    WgLayer a{};
    a.Z = bf16p(Z, "Z"); a.ldz = Z.stride(0); a.X = bf16p(X, "X"); a.ldx = X.stride(0);
    a.M = (int)M; a.N = (int)N; a.K = (int)K;
    a.alpha = (float)t[5].cast<double>(); a.lr = (float)t[6].cast<double>();
    auto chk2 = [&](const torch::Tensor& x, const char* nm) {
      TORCH_CHECK(x.is_cuda() && x.dim() == 2 && x.stride(1) == 1 && x.size(0) >= N && x.size(1) >= K, nm, " shape");
    };
    if (auto W = opt(t[7])) { chk2(*W, "W"); check_f32(*W, "W"); a.W = W->data_ptr<float>(); a.ldw = W->stride(0); }
    if (auto Wb = opt(t[8])) { chk2(*Wb, "Wb"); a.Wb = bf16p(*Wb, "Wb"); a.ldwb = Wb->stride(0); }
    if (auto G = opt(t[9])) { chk2(*G, "G"); check_f32(*G, "G"); a.G = G->data_ptr<float>(); a.ldg = G->stride(0); }
    if (auto b = opt(t[10])) { check_f32(*b, "bias"); TORCH_CHECK(b->numel() >= N, "bias"); a.bias = b->data_ptr<float>(); }
    if (auto bg = opt(t[11])) { check_f32(*bg, "bgrad"); TORCH_CHECK(bg->numel() >= N, "bgrad"); a.bgrad = bg->data_ptr<float>(); }
    if (t.size() >= 14) {  // split master: this step's hi words + the int16 remainders
      if (auto Wh = opt(t[12])) { chk2(*Wh, "Wh"); a.Wh = bf16p(*Wh, "Wh"); a.ldwh = Wh->stride(0); }
      if (auto Wl = opt(t[13])) {
        chk2(*Wl, "Wl");
        TORCH_CHECK(Wl->scalar_type() == torch::kInt16, "Wl must be int16");
        a.Wl = reinterpret_cast<uint16_t*>(Wl->data_ptr<int16_t>()); a.ldwl = Wl->stride(0);
      }
    }
    return a;
  };
  m.def("wgrad_sgd_multi", [wg_layer](py::list layers, int tile) {
    std::vector<WgLayer> v;
    for (py::handle it : layers) v.push_back(wg_layer(it));
    hip_ok(wgrad_sgd_multi(v.data(), (int)v.size(), cur_stream(), tile), "wgrad_sgd_multi");
  }, py::arg("layers"), py::arg("tile") = 0);
  // the fused input layer's operands (kernels/wide_input.hip, WideInArgs):
  // XG this step's rows in gradient-fragment order, contiguous [ceil(K/16)][2][16][32];
  // XF the next step's rows k-blocked, contiguous [ceil(K/32)][64][32]
  auto wide_in_args = [bf16p](torch::Tensor slabs, int64_t S, torch::Tensor H1, c10::optional<torch::Tensor> dzo,
                              torch::Tensor XG, torch::Tensor XF, torch::Tensor Wh, torch::Tensor Wl, torch::Tensor Wb,
                              torch::Tensor bias, double alpha, double lr, torch::Tensor Hn, int64_t M, int64_t N,
                              int64_t K) {
    auto rows2 = [&](const torch::Tensor& t, int64_t r, int64_t c, const char* nm) {
      TORCH_CHECK(t.is_cuda() && t.dim() == 2 && t.stride(1) == 1 && t.size(0) >= r && t.size(1) >= c, nm, " shape");
    };
    check_f32(slabs, "slabs");
    check_f32(bias, "bias");
    TORCH_CHECK(bias.numel() >= N, "bias");
    const int64_t tiles = (N + 63) / 64;
    TORCH_CHECK(slabs.numel() >= S * tiles * 4096, "slabs too small for S raw slices");
    rows2(H1, M, N, "H1"); rows2(Wh, N, K, "Wh"); rows2(Wl, N, K, "Wl");
    rows2(Wb, N, K, "Wb"); rows2(Hn, M, N, "Hn");
    TORCH_CHECK(Wl.scalar_type() == torch::kInt16, "Wl must be int16");
    TORCH_CHECK(XG.is_contiguous() && XG.numel() >= ((K + 15) / 16) * 1024, "XG: contiguous [K/16][2][16][32]");
    TORCH_CHECK(XF.is_contiguous() && XF.numel() >= ((K + 31) / 32) * 2048, "XF: contiguous [K/32][64][32]");
    WideInArgs a{};
    a.slabs = slabs.data_ptr<float>(); a.S = (int)S; a.tiles = (int)tiles; a.zalpha = 1.f; a.zbias = 0.f;
    a.H1 = bf16p(H1, "H1"); a.ldh1 = H1.stride(0);
    if (dzo) { rows2(*dzo, M, N, "dzo"); a.dzo = bf16p(*dzo, "dzo"); a.lddz = dzo->stride(0); }
    a.XG = bf16p(XG, "XG"); a.XF = bf16p(XF, "XF");
    a.Wh = bf16p(Wh, "Wh"); a.ldwh = Wh.stride(0);
    a.Wl = reinterpret_cast<uint16_t*>(Wl.data_ptr<int16_t>()); a.ldwl = Wl.stride(0);
    a.Wb = bf16p(Wb, "Wb"); a.ldwb = Wb.stride(0);
    a.bias = bias.data_ptr<float>(); a.alpha = (float)alpha; a.lr = (float)lr; a.falpha = 1.f;
    a.Hn = bf16p(Hn, "Hn"); a.ldhn = Hn.stride(0);
    a.M = (int)M; a.N = (int)N; a.K = (int)K; a.kq = (int)((((K + 7) / 8 + 31) / 32) * 32);
    return a;
  };
  m.def("wide_input_step", [wide_in_args](torch::Tensor slabs, int64_t S, torch::Tensor H1,
                                          c10::optional<torch::Tensor> dzo, torch::Tensor XG, torch::Tensor XF,
                                          torch::Tensor Wh, torch::Tensor Wl, torch::Tensor Wb, torch::Tensor bias,
                                          double alpha, double lr, torch::Tensor Hn, int64_t M, int64_t N, int64_t K) {
    const WideInArgs a = wide_in_args(slabs, S, H1, dzo, XG, XF, Wh, Wl, Wb, bias, alpha, lr, Hn, M, N, K);
    hip_ok(wide_input_step(a, cur_stream()), "wide_input_step");
  }, py::arg("slabs"), py::arg("S"), py::arg("H1"), py::arg("dzo"), py::arg("XG"), py::arg("XF"), py::arg("Wh"),
     py::arg("Wl"), py::arg("Wb"), py::arg("bias"), py::arg("alpha"), py::arg("lr"), py::arg("Hn"), py::arg("M"),
     py::arg("N"), py::arg("K"),
     "wide input layer: dZ_1 from raw dgrad slices, W_0 / b_0 SGD (split master), next step's H_1");
  m.def("wgrad_sgd_multi_in", [wg_layer, wide_in_args](py::list layers, torch::Tensor slabs, int64_t S,
                                                     torch::Tensor H1, c10::optional<torch::Tensor> dzo,
                                                     torch::Tensor XG, torch::Tensor XF, torch::Tensor Wh,
                                                     torch::Tensor Wl, torch::Tensor Wb, torch::Tensor bias,
                                                     double alpha, double lr, torch::Tensor Hn, int64_t M, int64_t N,
                                                     int64_t K) {
    std::vector<WgLayer> v;
    for (py::handle it : layers) v.push_back(wg_layer(it));
    const WideInArgs a = wide_in_args(slabs, S, H1, dzo, XG, XF, Wh, Wl, Wb, bias, alpha, lr, Hn, M, N, K);
    hip_ok(wgrad_sgd_multi_in(v.data(), (int)v.size(), a, cur_stream()), "wgrad_sgd_multi_in");
  }, py::arg("layers"), py::arg("slabs"), py::arg("S"), py::arg("H1"), py::arg("dzo"), py::arg("XG"), py::arg("XF"),
     py::arg("Wh"), py::arg("Wl"), py::arg("Wb"), py::arg("bias"), py::arg("alpha"), py::arg("lr"), py::arg("Hn"),
     py::arg("M"), py::arg("N"), py::arg("K"),
     "the update of the layers above the input layer (64 x 64 tiles) with the input layer's strips in the same launch");
  m.def("gemm_skinny_stamps", []() {
    std::vector<uint64_t> v(1024 * 5);
    hip_ok(gemm_skinny_read_stamps(v.data()), "gemm_skinny_read_stamps");
    return v;
  });
  m.def("gemm_skinny_set_stamping", &gemm_skinny_set_stamping);
  m.def("gemm_skinny_splits", &gemm_skinny_splits, py::arg("M"), py::arg("N"), py::arg("K"),
        py::arg("splits") = 0);
  m.def("hilo_split", [bf16p](torch::Tensor W, torch::Tensor hi, torch::Tensor lo) {
    // W [N x K] fp32 (row stride >= K) -> hi (bf16 words) / lo (int16) [>= N x >= K]
    check_f32(W, "W");
    TORCH_CHECK(W.dim() == 2 && W.stride(1) == 1 && hi.dim() == 2 && lo.dim() == 2 && hi.stride(1) == 1 &&
                lo.stride(1) == 1 && hi.size(0) >= W.size(0) && hi.size(1) >= W.size(1) &&
                lo.size(0) >= W.size(0) && lo.size(1) >= W.size(1), "hilo_split shapes");
    TORCH_CHECK(lo.scalar_type() == torch::kInt16, "lo must be int16");
    hip_ok(hilo_split(W.data_ptr<float>(), (int)W.size(0), (int)W.size(1), W.stride(0), bf16p(hi, "hi"),
                      hi.stride(0), reinterpret_cast<uint16_t*>(lo.data_ptr<int16_t>()), lo.stride(0),
                      cur_stream()), "hilo_split");
  });
  m.def("hilo_join", [bf16p](torch::Tensor hi, torch::Tensor lo, torch::Tensor W) {
    check_f32(W, "W");
    TORCH_CHECK(W.dim() == 2 && W.stride(1) == 1 && hi.dim() == 2 && lo.dim() == 2 && hi.stride(1) == 1 &&
                lo.stride(1) == 1 && hi.size(0) >= W.size(0) && hi.size(1) >= W.size(1) &&
                lo.size(0) >= W.size(0) && lo.size(1) >= W.size(1), "hilo_join shapes");
    TORCH_CHECK(lo.scalar_type() == torch::kInt16, "lo must be int16");
    hip_ok(hilo_join(bf16p(hi, "hi"), hi.stride(0), reinterpret_cast<const uint16_t*>(lo.data_ptr<int16_t>()),
                     lo.stride(0), (int)W.size(0), (int)W.size(1), W.data_ptr<float>(), W.stride(0), cur_stream()),
           "hilo_join");
  });
  m.def("sgd_cast", [bf16p](torch::Tensor W, c10::optional<torch::Tensor> G, int64_t N, int64_t K, double lr,
                           torch::Tensor Wb, c10::optional<torch::Tensor> WbT) {
    check_f32(W, "W");
    TORCH_CHECK(W.numel() >= N * K, "W too small");
    const float* g = nullptr;
    if (G) { check_f32(*G, "G"); TORCH_CHECK(G->numel() >= N * K, "G too small"); g = G->data_ptr<float>(); }
    TORCH_CHECK(Wb.dim() == 2 && Wb.size(0) >= N && Wb.size(1) >= K && Wb.stride(1) == 1, "Wb shape");
    uint16_t* t = nullptr; int64_t ldt = 0;
    if (WbT) { TORCH_CHECK(WbT->dim() == 2 && WbT->size(0) >= K && WbT->size(1) >= N && WbT->stride(1) == 1, "WbT shape");
               t = bf16p(*WbT, "WbT"); ldt = WbT->stride(0); }
    hip_ok(sgd_cast(W.data_ptr<float>(), g, (int)N, (int)K, (float)lr, bf16p(Wb, "Wb"), Wb.stride(0), t, ldt,
                    cur_stream()), "sgd_cast");
  });

  // ---- fused MLP -----------------------------------------------------------
  m.def("mlp_stamps", []() {
    std::vector<uint64_t> v(kMaxStamps);
    hip_ok(mlp_read_stamps(v.data()), "mlp_read_stamps");
    return v;
  });
  m.def("mlp_set_stamping", [](bool on) {
    mlp_set_stamping(on);
    mlp_set_stamping_fast(on);
    mlp_set_stamping_xact(on);
  });
  m.def("mlp_stamps_xact", []() {
    std::vector<uint64_t> v(kMaxStamps);
    hip_ok(mlp_read_stamps_xact(v.data()), "mlp_read_stamps_xact");
    return v;
  });
  m.def("mlp_stamps_fast", []() {
    std::vector<uint64_t> v(kMaxStamps);
    hip_ok(mlp_read_stamps_fast(v.data()), "mlp_read_stamps_fast");
    return v;
  });
  m.def("mlp_persist_supported", [](const std::vector<int64_t>& desc) {
    return mlp_persist_supported(desc_from_list(desc));
  });
  m.def("wgrad_rowblk_plan", [](const std::vector<int>& N, const std::vector<int>& K, int groups) {
    TORCH_CHECK(N.size() == K.size() && !N.empty() && N.size() <= 8, "wgrad_rowblk_plan: 1-8 layers");
    TORCH_CHECK(groups >= 1 && groups <= 256, "wgrad_rowblk_plan: 1-256 groups");
    std::vector<int> st(257);
    const int g = wgrad_rowblk_plan(N.data(), K.data(), (int)N.size(), groups, st.data());
    st.resize(g + 1);
    return st;
  }, py::arg("N"), py::arg("K"), py::arg("groups"),
        "row-block update: cost-balanced workgroup runs (unit starts) for layers (N, K) in launch order");
  m.def("mlp_persist_xbuf_granules", []() { return mlp_persist_xbuf_granules(); });
  m.def("mlp_persist_stamps", []() {
    std::vector<uint64_t> v(4 * 8 * 8);
    hip_ok(mlp_persist_read_stamps(v.data()), "mlp_persist_read_stamps");
    return v;
  });
  m.def("mlp_persist_set_stamping", [](bool on) { mlp_persist_set_stamping(on); });
  m.def("mlp_persist_set_stamp_window", [](int first_step) { mlp_persist_set_stamp_window(first_step); },
        "stamp steps first_step .. first_step + 7 of a launch (< 0: off)");
  m.def("gram_table", [](torch::Tensor Xs, torch::Tensor Xc, int64_t nb, int64_t B, int64_t K) {
    // Xs: one source [rows][ld] (-> T [nb][64][64]) or [nsrc][rows][ld]
    // (-> T [nb][nsrc][64][64]); Xc [rows][ld]: the batches the table is for
    check_cuda_strided(Xs, "Xs");
    check_cuda_strided(Xc, "Xc");
    TORCH_CHECK(Xs.scalar_type() == torch::kFloat32 && Xc.scalar_type() == torch::kFloat32,
                "gram_table: float32 operands");
    TORCH_CHECK(Xs.dim() == 2 || Xs.dim() == 3, "Xs: [rows][ld] or [nsrc][rows][ld]");
    TORCH_CHECK(Xc.dim() == 2 && Xc.stride(1) == 1 && Xs.stride(-1) == 1, "rows must be contiguous");
    TORCH_CHECK(nb >= 1 && B >= 1 && B <= 64 && K >= 1, "gram_table: nb >= 1, 1 <= B <= 64, K >= 1");
    const int64_t rows = nb * B;
    const int64_t nsrc = Xs.dim() == 3 ? Xs.size(0) : 1;
    TORCH_CHECK(Xs.size(-2) >= rows && Xc.size(0) >= rows && Xs.size(-1) >= K && Xc.size(1) >= K,
                "gram_table: operands hold fewer than nb * B rows or K columns");
    TORCH_CHECK(Xs.get_device() == Xc.get_device(), "gram_table: operands on one GPU");
    const int64_t sstride = Xs.dim() == 3 ? Xs.stride(0) : 0;
    auto T = torch::empty(Xs.dim() == 3 ? std::vector<int64_t>{nb, nsrc, 64, 64} : std::vector<int64_t>{nb, 64, 64},
                          Xc.options());
    hip_ok(gram_table(Xs.data_ptr<float>(), sstride, Xs.stride(-2), Xc.data_ptr<float>(), Xc.stride(0), (int)nb,
                      (int)B, (int)K, (int)nsrc, T.data_ptr<float>(), cur_stream()),
           "gram_table");
    return T;
  }, py::arg("Xs"), py::arg("Xc"), py::arg("nb"), py::arg("B"), py::arg("K"),
     "Gram tables of the persistent step's Gram form (kernels/gram.hip; engine/gram.py is the "
     "float64 torch oracle)");
  m.def("mlp_persist_set_pkx_helpers", [](int h) { mlp_persist_set_pkx_helpers(h); }, py::arg("helpers"),
        "pkx dW1 helper blocks per layer-1 block: -1 default (3 from 4 replicas on), 0, 1 or 3");
  m.def("mlp_persist_set_pkx_l1push", [](int v) { mlp_persist_set_pkx_l1push(v); }, py::arg("mode"),
        "pkx dZ1 row pushes to the peers: 1 from the layer-1 owner blocks, 0 from the chains, -1 default");
#ifdef HIPDSML_MEASURE
  m.def("mlp_persist_push_stamps", []() {
    std::vector<uint64_t> v(8 * 4);
    hip_ok(mlp_persist_read_push_stamps(v.data()), "mlp_persist_read_push_stamps");
    return v;
  });
  m.def("mlp_persist_set_hop", [](double us) { mlp_persist_set_hop((int)(us * 100.0 + 0.5)); }, py::arg("us"),
        "measurement builds: every cross-replica hop of the mirror mode becomes usable `us` after "
        "its publication (0 off)");
#endif
  m.def("mlp_persist_set_probe", [](int mode) { mlp_persist_set_probe(mode); },
        "testing only: 0 off; 1 peers' dZ1 rows taken as arrived (lone-replica probe of the Gram "
        "forms); 2 mirror: every push loops back into this replica's own buffer in the peer's "
        "source slot (N-replica step against N - 1 copies of itself)");
  m.def("mlp_persist_set_jitter", [](int ticks) { mlp_persist_set_jitter(ticks); },
        "testing only: every block of the single-replica persistent step sleeps a pseudo-random "
        "0..ticks x 64 cycles before its hand-offs (0 = off)");
  m.def("mlp_plan", [](const std::vector<int64_t>& desc) {
    const MlpDesc d = desc_from_list(desc);
    const MlpLaunchCfg c = mlp_plan_first_layer(d);
    return py::make_tuple(c.kchunk, c.nsplit, mlp_wgrad_tiles(d), mlp_rowchain_fits(d));
  });
  m.def("mlp_eval", [](const std::vector<int64_t>& desc, torch::Tensor X, torch::Tensor labels,
                       int64_t row0, torch::Tensor P, torch::Tensor ws, torch::Tensor slab,
                       torch::Tensor stats) {
    const MlpDesc d = desc_from_list(desc);
    check_f32(X, "X"); check_f32(P, "P"); check_f32(slab, "slab"); check_f32(stats, "stats");
    check_f32(ws, "ws"); check_cuda(labels, "labels");
    TORCH_CHECK(labels.scalar_type() == torch::kInt32, "labels must be int32");
    TORCH_CHECK(X.dim() == 2 && X.size(1) % 4 == 0 && X.size(1) >= d.dims[0], "bad X");
    TORCH_CHECK(row0 >= 0 && row0 + d.batch <= X.size(0) && row0 + d.batch <= labels.numel(),
                "eval rows out of range");
    TORCH_CHECK(P.numel() >= layout_param_end(d), "params too small");
    const MlpLaunchCfg c = mlp_plan_first_layer(d);
    TORCH_CHECK(slab.numel() >= (int64_t)c.nsplit * d.batch * d.dims[1], "slab too small");
    TORCH_CHECK(d.lds_floats * 4 <= 160 * 1024, "model too wide for the fused row chain");
    mlp_eval(d, X.data_ptr<float>(), X.size(1), labels.data_ptr<int32_t>(), row0,
             P.data_ptr<float>(), ws.data_ptr<float>(), slab.data_ptr<float>(),
             stats.data_ptr<float>(), cur_stream());
  });
  // Forward on the fused kernels with the logits kept: returns a [batch x C]
  // view into ws (ws must cover the full layout of `desc`).  The RunForward RPC.
  m.def("mlp_forward_logits", [](const std::vector<int64_t>& desc, torch::Tensor X,
                                 torch::Tensor labels, int64_t row0, torch::Tensor P,
                                 torch::Tensor ws, torch::Tensor slab, torch::Tensor stats) {
    const MlpDesc d = desc_from_list(desc);
    check_f32(X, "X"); check_f32(P, "P"); check_f32(slab, "slab"); check_f32(stats, "stats");
    check_f32(ws, "ws"); check_cuda(labels, "labels");
    TORCH_CHECK(labels.scalar_type() == torch::kInt32, "labels must be int32");
    TORCH_CHECK(X.dim() == 2 && X.size(1) % 4 == 0 && X.size(1) >= d.dims[0], "bad X");
    TORCH_CHECK(row0 >= 0 && row0 + d.batch <= X.size(0) && row0 + d.batch <= labels.numel(),
                "rows out of range");
    TORCH_CHECK(P.numel() >= layout_param_end(d), "params too small");
    TORCH_CHECK(ws.numel() >= layout_ws_end(d), "workspace too small for the layout");
    TORCH_CHECK(stats.numel() >= 3, "stats must hold 3 floats");
    const MlpLaunchCfg c = mlp_plan_first_layer(d);
    TORCH_CHECK(slab.numel() >= (int64_t)c.nsplit * d.batch * d.dims[1], "slab too small");
    TORCH_CHECK(d.lds_floats * 4 <= 160 * 1024, "model too wide for the fused row chain");
    mlp_eval(d, X.data_ptr<float>(), X.size(1), labels.data_ptr<int32_t>(), row0,
             P.data_ptr<float>(), ws.data_ptr<float>(), slab.data_ptr<float>(),
             stats.data_ptr<float>(), cur_stream(), true);
    const int C = d.dims[d.nlayers];
    return ws.narrow(0, d.dz_off[d.nlayers], (int64_t)d.batch * C).view({d.batch, C});
  });

  py::class_<PyMlpRunner>(m, "MlpRunner")
      .def(py::init<const std::vector<int64_t>&, torch::Tensor, torch::Tensor, torch::Tensor,
                    torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor,
                    torch::Tensor, float, float, float, uintptr_t, bool>(),
           py::arg("desc"), py::arg("X"), py::arg("labels"), py::arg("P"), py::arg("G"),
           py::arg("V"), py::arg("ws"), py::arg("slab"), py::arg("ctr"), py::arg("stats"),
           py::arg("lr"), py::arg("momentum"), py::arg("weight_decay"), py::arg("stream") = 0,
           py::arg("follow_torch") = false)
      .def_property_readonly("follows_torch", [](PyMlpRunner& s) { return s.follow; })
      .def("step", &PyMlpRunner::step, py::arg("n") = 1, py::arg("join") = true)
      .def("fwd_bwd", &PyMlpRunner::fwd_bwd)
      .def("update", &PyMlpRunner::update)
      .def("capture", &PyMlpRunner::capture, py::arg("steps"), py::arg("capture_comm") = true)
      .def("replay", &PyMlpRunner::replay, py::arg("times") = 1, py::arg("steps") = 0)
      .def("captured", [](PyMlpRunner& s, int steps) { return s.r->captured(steps); },
           py::arg("steps") = 0)
      .def("synchronize", &PyMlpRunner::synchronize)
      .def("join_into_torch", &PyMlpRunner::join_into_torch)
      .def("stream_handle", &PyMlpRunner::stream_handle)
      .def("graph_steps", [](PyMlpRunner& s) { return s.r->graph_steps(); })
      .def("set_lr", [](PyMlpRunner& s, float lr) { s.r->set_lr(lr); })
      .def("set_world_size", [](PyMlpRunner& s, int n) { s.r->set_world_size(n); })
      .def("set_comm", [](PyMlpRunner& s, PyComm* c, int algo, int64_t chunk) {
        s.r->set_comm(c ? c->c.get() : nullptr, algo, chunk);
      }, py::arg("comm"), py::arg("algo") = 0, py::arg("chunk_bytes") = 1 << 20)
      .def("set_exchange", [](PyMlpRunner& s, PeerExchange* x) { s.r->set_exchange(x); },
           py::arg("exchange").none(true), py::keep_alive<1, 2>())
      .def("set_act_exchange", [](PyMlpRunner& s, PeerExchange* x, torch::Tensor Xall,
                                  int64_t xstride, int waves) {
        check_f32(Xall, "Xall");
        TORCH_CHECK(Xall.is_contiguous(), "Xall must be contiguous");
        TORCH_CHECK(x == nullptr || Xall.numel() >= (int64_t)x->nranks() * xstride,
                    "Xall holds fewer than nranks shards");
        s.r->set_act_exchange(x, Xall.data_ptr<float>(), xstride, waves);
        s.keep_xact_in = Xall;
      }, py::arg("exchange").none(true), py::arg("Xall"), py::arg("xstride"), py::arg("waves") = 0,
           py::keep_alive<1, 2>())
      .def("set_persist", [](PyMlpRunner& s, c10::optional<torch::Tensor> xbuf,
                             c10::optional<torch::Tensor> err, double timeout_ms, PeerExchange* x,
                             int algo) {
        if (!xbuf) { s.r->set_persist(nullptr, nullptr, 0.0); return; }
        check_cuda(*xbuf, "xbuf");
        TORCH_CHECK(xbuf->scalar_type() == torch::kInt64 &&
                    xbuf->numel() >= mlp_persist_xbuf_granules(), "xbuf: int64[",
                    mlp_persist_xbuf_granules(), "]");
        TORCH_CHECK(err && err->is_cuda() && err->scalar_type() == torch::kInt32 && err->numel() >= 1,
                    "err: int32[1] on the GPU");
        s.keep_xbuf = *xbuf;
        s.keep_err = *err;
        s.r->set_persist(reinterpret_cast<uint64_t*>(xbuf->data_ptr<int64_t>()),
                         reinterpret_cast<uint32_t*>(err->data_ptr<int32_t>()), timeout_ms, x, algo);
      }, py::arg("xbuf").none(true), py::arg("err") = py::none(), py::arg("timeout_ms") = 2000.0,
         py::arg("exchange") = nullptr, py::arg("algo") = 0, py::keep_alive<1, 5>())
      .def_static("persist_xchg_size", [](int n, int algo) {
        return py::make_tuple(px_half(n, algo), px_ntiles(n, algo)); }, py::arg("n"), py::arg("algo") = 0,
                  "(half_floats, ntiles) of the persistent step's replica exchange at n ranks "
                  "(algo 0: one-shot, 1: two-shot)")
      .def("persist_active", [](PyMlpRunner& s) { return s.r->persist_active(); })
      .def("persist_failed", [](PyMlpRunner& s) { return s.r->persist_failed(); },
           "a persistent launch gave up on a hand-off (valid after a sync; no device copy)")
      .def("clear_persist_error", [](PyMlpRunner& s) { s.r->clear_persist_error(); })
      .def("set_persist_gram", [](PyMlpRunner& s, torch::Tensor g) {
        check_f32(g, "gram");
        TORCH_CHECK(g.is_contiguous() && g.numel() >= (int64_t)s.r->desc().nbatches * 64 * 64,
                    "gram: contiguous float[nbatches][64][64]");
        TORCH_CHECK((reinterpret_cast<uintptr_t>(g.data_ptr<float>()) & 15) == 0, "gram: 16-B aligned");
        s.keep_gram = g;
        s.r->set_persist_gram(g.data_ptr<float>(), g.numel());
      }, py::arg("gram"),
           "single-replica persistent step: the per-batch Gram table G1T[b][m'][m] = "
           "X_{b-1}[m'] . X_b[m] + 1 (trainer._gram_table)")
      .def("set_persist_carry", [](PyMlpRunner& s, bool c) { s.r->set_persist_carry(c); }, py::arg("carry"))
      .def("set_persist_xall", [](PyMlpRunner& s, torch::Tensor x, int64_t stride) {
        check_f32(x, "xsw");
        TORCH_CHECK(x.is_contiguous() && stride > 0 && stride % 4 == 0, "xsw: contiguous, stride % 4 == 0");
        TORCH_CHECK((reinterpret_cast<uintptr_t>(x.data_ptr<float>()) & 15) == 0, "xsw: 16-B aligned");
        s.keep_xall = x;
        s.r->set_persist_xall(x.data_ptr<float>(), stride, x.numel());
      }, py::arg("xsw"), py::arg("stride"),
           "exchange-free data-parallel persistent step (pkx): every replica's input shard in "
           "MFMA fragment order (parallel/xchg.py swizzle_inputs), replica r at r * stride floats")
      .def("release_xall", [](PyMlpRunner& s) {
        TORCH_CHECK(s.r->exchange_mode() != 2, "release_xall: the activation exchange still reads Xall");
        s.r->set_persist_xall(nullptr, 0, 0);
        s.keep_xall = torch::Tensor();
        s.keep_xact_in = torch::Tensor();
      }, "drop the runner's references to the replicated input shards (neither pkx nor xact "
         "runs any more; the next pkx launch would refuse to start without new ones)")
      .def("persist_carry", [](PyMlpRunner& s) { return s.r->persist_carry(); },
           "the hand-off buffer holds the last launch's pipeline state (next partials + correction)")
      .def("exchange_active", [](PyMlpRunner& s) { return s.r->exchange_active(); })
      .def("exchange_mode", [](PyMlpRunner& s) { return s.r->exchange_mode(); })
      .def("plan", [](PyMlpRunner& s) {
        const MlpLaunchCfg c = s.r->cfg();
        return py::make_tuple(c.kchunk, c.nsplit);
      });

  // ---- multi-ring schedule (pure index math; CPU-testable) -----------------
  m.def("ring_schedule", [](int n, int rank, int64_t count, int64_t align, int64_t chunk,
                            int max_rings) {
    py::list steps;
    for (const auto& g : ring_schedule(n, rank, count, align, chunk, max_rings)) {
      py::list ops;
      for (const auto& x : g)
        ops.append(py::make_tuple(x.ring, x.send_peer, x.send_off, x.send_len, x.recv_peer,
                                  x.recv_off, x.recv_len, x.reduce));
      steps.append(ops);
    }
    return steps;
  }, py::arg("n"), py::arg("rank"), py::arg("count"), py::arg("align") = 4,
     py::arg("chunk") = 0, py::arg("max_rings") = 0);
  m.def("ring_pipeline", [](int n, int rank, int64_t count, int64_t align, int64_t chunk,
                            int max_rings) {
    py::list out;
    for (const auto& d : ring_pipeline(ring_schedule(n, rank, count, align, chunk, max_rings)))
      out.append(py::make_tuple(d.wait_reduce, d.slot, d.slot_free));
    return out;
  }, py::arg("n"), py::arg("rank"), py::arg("count"), py::arg("align") = 4,
     py::arg("chunk") = 0, py::arg("max_rings") = 0,
     "per group of ring_schedule: (wait_reduce, slot, slot_free) of the two-stream pipelined ring");
  m.def("directed_rings", &directed_rings, py::arg("n"), py::arg("max_rings") = 0);

  // ---- xGMI peer exchange (gradient all-reduce fused into K_C) -------------
  m.def("mlp_wgrad_tiles", [](const std::vector<int64_t>& desc) {
    return mlp_wgrad_tiles(desc_from_list(desc));
  });
  m.def("mlp_xact_payload", [](const std::vector<int64_t>& desc) {
    return mlp_xact_payload(desc_from_list(desc));
  });
  m.def("mlp_xact_supported", [](const std::vector<int64_t>& desc) {
    return mlp_xact_supported(desc_from_list(desc));
  });
  py::class_<PeerExchange>(m, "PeerExchange")
      .def(py::init<int, int64_t, int>(), py::arg("device"), py::arg("half_floats"),
           py::arg("ntiles"))
      .def("ipc_handle", [](PeerExchange& x) {
        const auto v = x.ipc_handle();
        return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
      })
      .def("connect_ipc", [](PeerExchange& x, int rank, const std::vector<py::bytes>& hs) {
        std::vector<std::vector<uint8_t>> v;
        for (const auto& h : hs) {
          std::string t = h;
          v.emplace_back(t.begin(), t.end());
        }
        x.connect_ipc(rank, v);
      })
      .def("connect_local", &PeerExchange::connect_local)
      .def("reset", [](PeerExchange& x) { x.reset(cur_stream()); })
      // Probe/debug only: preset every flag of this exchange (e.g. to a value
      // no step reaches, so a lone replica measures its kernels without waits).
      .def("fill_flags", [](PeerExchange& x, uint64_t v) {
        std::vector<uint64_t> h((size_t)x.ntiles(), v);
        DSML_HIP_CHECK(hipMemcpy(x.flags(), h.data(), h.size() * sizeof(uint64_t),
                                 hipMemcpyHostToDevice));
      })
      .def("error", [](PeerExchange& x) {
        py::gil_scoped_release nogil;
        return x.error(cur_stream());
      })
      .def("set_timeout_ms", &PeerExchange::set_timeout_ms)
      .def("allreduce_", [](PeerExchange& x, torch::Tensor t, int algo) {
        check_f32(t, "tensor");
        x.allreduce(t.data_ptr<float>(), t.data_ptr<float>(), t.numel(), cur_stream(), algo);
        return t;
      }, py::arg("t"), py::arg("algo") = 0)
      .def("allreduce", [](PeerExchange& x, torch::Tensor in, torch::Tensor out, int algo) {
        check_f32(in, "in");
        check_f32(out, "out");
        TORCH_CHECK(in.numel() == out.numel(), "in/out size mismatch");
        x.allreduce(in.data_ptr<float>(), out.data_ptr<float>(), in.numel(), cur_stream(), algo);
        return out;
      }, py::arg("in"), py::arg("out"), py::arg("algo") = 0)
      .def_property_readonly("nranks", &PeerExchange::nranks)
      .def_property_readonly("rank", &PeerExchange::rank)
      .def_property_readonly("ntiles", &PeerExchange::ntiles)
      .def_property_readonly("half", &PeerExchange::half)
      .def_property_readonly("memory_kind", &PeerExchange::memory_kind)
      .def_property_readonly("connected", &PeerExchange::connected);

  // ---- RCCL ----------------------------------------------------------------
  m.def("rccl_unique_id", []() {
    const auto v = rccl_unique_id();
    return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
  });
  py::class_<PyComm>(m, "RcclComm")
      .def(py::init<py::bytes, int, int, int, bool>(), py::arg("uid"), py::arg("rank"),
           py::arg("nranks"), py::arg("device"), py::arg("blocking") = true)
      .def_property_readonly("rank", [](PyComm& s) { return live(s)->rank(); })
      .def_property_readonly("nranks", [](PyComm& s) { return live(s)->nranks(); })
      .def("allreduce_", [](PyComm& s, torch::Tensor t, int op) {
        check_cuda(t, "t");
        live(s)->allreduce(t.data_ptr(), t.numel(), dtype_of(t), op, cur_stream());
      }, py::arg("t"), py::arg("op") = 0)
      .def("ring_allreduce_", [](PyComm& s, torch::Tensor t, int op, int64_t chunk_bytes,
                                 int max_rings, int pipe) {
        check_cuda(t, "t");
        TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, "tensor must be 16 B aligned");
        live(s)->ring_allreduce(t.data_ptr(), t.numel(), dtype_of(t), op, chunk_bytes, cur_stream(),
                            max_rings, pipe);
      }, py::arg("t"), py::arg("op") = 0, py::arg("chunk_bytes") = 1 << 20,
         py::arg("max_rings") = 0, py::arg("pipe") = -1,
         "pipe: 1 pipelined schedule, 0 single-stream, -1 the communicator's default")
      .def("set_ring_pipeline", [](PyComm& s, int mode) { live(s)->set_ring_pipeline(mode); }, py::arg("mode"))
      .def_property_readonly("ring_pipeline", [](PyComm& s) { return live(s)->pipeline_mode(); })
      .def("reserve_ring", [](PyComm& s, int64_t count, int64_t chunk_bytes, int max_rings) {
        live(s)->reserve_ring(count, kF32, chunk_bytes, max_rings);
      }, py::arg("count"), py::arg("chunk_bytes") = 1 << 20, py::arg("max_rings") = 0,
         "size the fp32 ring all-reduce scratch for `count` elements up front")
      .def("broadcast_", [](PyComm& s, torch::Tensor t, int root) {
        check_cuda(t, "t");
        live(s)->broadcast(t.data_ptr(), t.numel(), dtype_of(t), root, cur_stream());
      })
      .def("allgather_", [](PyComm& s, torch::Tensor t) {
        check_cuda(t, "t");
        TORCH_CHECK(t.is_contiguous() && t.numel() % live(s)->nranks() == 0,
                    "allgather_: contiguous, nranks equal parts");
        live(s)->allgather(t.data_ptr(), t.numel() / live(s)->nranks(), dtype_of(t), cur_stream());
      }, py::arg("t"), "in-place all-gather: rank r contributes part r of t")
      .def("send", [](PyComm& s, torch::Tensor t, int peer) {
        check_cuda(t, "t");
        live(s)->send(t.data_ptr(), t.numel(), dtype_of(t), peer, cur_stream());
      })
      .def("recv_", [](PyComm& s, torch::Tensor t, int peer) {
        check_cuda(t, "t");
        live(s)->recv(t.data_ptr(), t.numel(), dtype_of(t), peer, cur_stream());
      })
      .def("barrier", [](PyComm& s) {
        hipStream_t st = cur_stream();
        py::gil_scoped_release nogil;
        live(s)->barrier(st);
      })
      .def("abort", [](PyComm& s) { if (s.c) s.c->abort(); })
      .def("destroy", [](PyComm& s) {
        py::gil_scoped_release nogil;  // ncclCommDestroy (or the aborted comm's buffers) freed now
        s.c.reset();
      }, "free the communicator now (a destroyed comm raises on any further use)")
      .def("async_error", [](PyComm& s) { return s.c ? s.c->async_error() : std::string("aborted"); })
      .def_property_readonly("aborted", [](PyComm& s) { return !s.c || s.c->aborted(); });

  // ---- device runtime (arena / copy engine / stream table) ------------------
  py::class_<DeviceArena>(m, "DeviceArena")
      .def(py::init<int, uint64_t, uint64_t>(), py::arg("device"), py::arg("size"),
           py::arg("base_addr") = DeviceArena::kBaseAddr)
      .def_property_readonly("min_addr", &DeviceArena::min_addr)
      .def_property_readonly("max_addr", &DeviceArena::max_addr)
      .def_property_readonly("size", &DeviceArena::size)
      .def("contains", &DeviceArena::contains)
      .def("ptr", [](DeviceArena& a, uint64_t addr, uint64_t n) {
        try { return reinterpret_cast<uintptr_t>(a.translate(addr, n)); }
        catch (const std::out_of_range& e) { throw py::index_error(e.what()); }
      })
      .def("record_extent", &DeviceArena::record_extent)
      .def("extent", &DeviceArena::extent)
      .def("reduce", [](DeviceArena& a, uint64_t dst, uint64_t src, uint64_t nbytes, int dtype,
                        int op) {
        const uint64_t es = dtype == kF32 || dtype == kI32 ? 4 : (dtype == kU8 ? 1 : 2);
        void* d = nullptr; void* sp = nullptr;
        try { d = a.translate(dst, nbytes); sp = a.translate(src, nbytes); }
        catch (const std::out_of_range& e) { throw py::index_error(e.what()); }
        TORCH_CHECK(nbytes % es == 0, "nbytes not a multiple of the element size");
        hipStream_t s = nullptr;
        hip_ok(reduce_inplace(d, sp, (int64_t)(nbytes / es), dtype, op, s), "reduce_inplace");
        hip_ok(hipStreamSynchronize(s), "sync");
      });
  py::class_<CopyEngine>(m, "CopyEngine")
      .def(py::init<int, size_t>(), py::arg("device"), py::arg("staging_bytes") = 16u << 20)
      .def("h2d", [](CopyEngine& c, DeviceArena& a, uint64_t addr, py::bytes data) {
        std::string s = data;
        void* dst;
        try { dst = a.translate(addr, s.size()); }
        catch (const std::out_of_range& e) { throw py::index_error(e.what()); }
        py::gil_scoped_release nogil;
        c.h2d(dst, s.data(), s.size());
        a.record_extent(addr, s.size());
      })
      .def("d2h", [](CopyEngine& c, DeviceArena& a, uint64_t addr, uint64_t n) {
        const void* src;
        try { src = a.translate(addr, n); }
        catch (const std::out_of_range& e) { throw py::index_error(e.what()); }
        std::string out(n, '\0');
        {
          py::gil_scoped_release nogil;
          c.d2h(out.data(), src, n);
        }
        return py::bytes(out);
      })
      .def("d2d", [](CopyEngine& c, DeviceArena& a, uint64_t dst, uint64_t src, uint64_t n) {
        void* d; const void* s;
        try { d = a.translate(dst, n); s = a.translate(src, n); }
        catch (const std::out_of_range& e) { throw py::index_error(e.what()); }
        py::gil_scoped_release nogil;
        c.d2d(d, s, n);
      })
      .def_property_readonly("bytes_h2d", &CopyEngine::bytes_h2d)
      .def_property_readonly("bytes_d2h", &CopyEngine::bytes_d2h);
  py::class_<StreamTable>(m, "StreamTable")
      .def(py::init<DeviceArena*, CopyEngine*>(), py::keep_alive<1, 2>(), py::keep_alive<1, 3>())
      .def("begin_send", &StreamTable::begin_send)
      .def("begin_receive", [](StreamTable& t, uint64_t id, uint64_t addr, uint64_t n, uint32_t src) {
        try { t.begin_receive(id, addr, n, src); }
        catch (const std::out_of_range& e) { throw py::index_error(e.what()); }
        catch (const std::invalid_argument& e) { throw py::key_error(e.what()); }
      })
      .def("push_chunk", [](StreamTable& t, uint64_t id, py::bytes data) {
        std::string s = data;
        py::gil_scoped_release nogil;
        return t.push_chunk(id, s.data(), s.size());
      })
      .def("finish", &StreamTable::finish)
      .def("status", [](StreamTable& t, uint64_t id) { return (int)t.status(id); })
      .def("read_send_buffer", [](StreamTable& t, uint64_t id) {
        std::vector<uint8_t> v;
        try { v = t.read_send_buffer(id); }
        catch (const std::invalid_argument& e) { throw py::key_error(e.what()); }
        return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
      })
      .def("erase", &StreamTable::erase)
      .def("__len__", &StreamTable::size);

  // roctx ranges / markers (shown by rocprofv3 --marker-trace; no-ops otherwise).
  m.def("roctx_push", [](const std::string& name) { return roctxRangePushA(name.c_str()); });
  m.def("roctx_pop", []() { return roctxRangePop(); });
  m.def("roctx_mark", [](const std::string& name) { roctxMarkA(name.c_str()); });
  // A stream on a hardware queue of its own.  HIP hands ordinary new streams
  // the least-used of its GPU_MAX_HW_QUEUES (4) queues once they all exist; a
  // stream created with a CU mask always gets a fresh queue.  In-process
  // replicas that spin on each other (xGMI exchange tests) need exactly that:
  // two of them sharing a queue would serialise, the later one never starting.
  // The mask covers every CU (no partitioning); the stream lives until
  // stream_destroy.
  m.def("dedicated_stream", [](int device) {
    hip_ok(hipSetDevice(device), "hipSetDevice");
    hipDeviceProp_t p;
    hip_ok(hipGetDeviceProperties(&p, device), "hipGetDeviceProperties");
    std::vector<uint32_t> mask((size_t)(p.multiProcessorCount + 31) / 32, 0xffffffffu);
    hipStream_t st = nullptr;
    hip_ok(hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()),
           "hipExtStreamCreateWithCUMask");
    return reinterpret_cast<uintptr_t>(st);
  });
  m.def("stream_destroy", [](uintptr_t h) {
    hip_ok(hipStreamDestroy(reinterpret_cast<hipStream_t>(h)), "hipStreamDestroy");
  });
  m.def("device_count", []() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    return n;
  });
}
