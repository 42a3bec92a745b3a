// pybind11 bindings: the Engine (runtime) plus raw-pointer op entry points used by the kernel
// numerics tests (torch tensors pass data_ptr() and torch.cuda.current_stream().cuda_stream).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>

#include "comm.h"
#include "rccl_comm.h"
#include "engine.h"
#include "grammar.h"
#include "ops.h"

namespace py = pybind11;
using namespace aios;

namespace aios {
double bench_launch_chain(int n_kernels, int blocks, int use_graph, int reps);
double bench_stream_read(size_t bytes, int nbuf, int wg_per_cu, int u, int threads, int reps);
double bench_stream_read_part(size_t bytes, int nbuf, int mode, int threads, int reps);
}

namespace {

hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

// split-K workspace for GEMM calls from Python (tests / tools): grown on demand, never freed;
// tickets zeroed once (the kernel's last arriver re-arms them)
struct GemmWs {
  float* ws = nullptr;
  size_t bytes = 0;
  int* cnt = nullptr;
  int cnt_len = 0;
};
GemmWs& gemm_ws(int M, int N) {
  static GemmWs g;
  const size_t need = gemm_skinny_ws_bytes(std::min(M, 64), N);
  const int need_cnt = gemm_skinny_cnt_len(N);
  if (need > g.bytes) {
    HIP_CHECK(hipDeviceSynchronize());
    if (g.ws) HIP_CHECK(hipFree(g.ws));
    HIP_CHECK(hipMalloc(&g.ws, need));
    g.bytes = need;
  }
  if (need_cnt > g.cnt_len) {
    HIP_CHECK(hipDeviceSynchronize());
    if (g.cnt) HIP_CHECK(hipFree(g.cnt));
    HIP_CHECK(hipMalloc(&g.cnt, need_cnt * 4));
    HIP_CHECK(hipMemset(g.cnt, 0, need_cnt * 4));
    g.cnt_len = need_cnt;
  }
  return g;
}

// Owning device matrix in the repacked layout (tests / tools)
struct PyQMatrix {
  QWeight w{};
  void* buf = nullptr;
  size_t bytes = 0;
  PyQMatrix(int qt, int rows, int cols, py::buffer raw) {
    py::buffer_info bi = raw.request();
    const size_t nbytes = (size_t)bi.size * bi.itemsize;
    // engine-less allocation mirroring Engine::alloc_qmat
    EngineConfig cfg;
    cfg.n_layers = 0;
    (void)cfg;
    const int be = (qt == QT_Q4_K || qt == QT_Q5_K || qt == QT_Q6_K) ? 256 : ((qt == QT_F16 || qt == QT_BF16) ? 1 : 32);
    const size_t nb = (size_t)rows * (cols / be);
    size_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
    switch (qt) {
      case QT_Q4_K: s0 = nb * 128; s1 = nb * 16; break;
      case QT_Q5_K: s0 = nb * 128; s1 = nb * 16; s2 = nb * 32; break;
      case QT_Q6_K: s0 = nb * 128; s1 = nb * 64; s2 = nb * 16; s3 = nb * 2; break;
      case QT_Q4_0: s0 = nb * 16; s1 = nb * 2; break;
      case QT_Q8_0: s0 = nb * 32; s1 = nb * 2; break;
      case QT_F16:
      case QT_BF16: s0 = nb * 2; break;
      default: throw std::runtime_error("QMatrix: unsupported type");
    }
    auto al = [](size_t x) { return (x + 255) / 256 * 256; };
    const size_t o1 = al(s0), o2 = o1 + al(s1), o3 = o2 + al(s2);
    bytes = o3 + al(s3) + 64;
    HIP_CHECK(hipMalloc(&buf, bytes));
    uint8_t* base = (uint8_t*)buf;
    w.qtype = qt;
    w.rows = rows;
    w.cols = cols;
    w.p0 = base;
    w.p1 = s1 ? base + o1 : nullptr;
    w.p2 = s2 ? base + o2 : nullptr;
    w.p3 = s3 ? base + o3 : nullptr;
    void* staging = nullptr;
    HIP_CHECK(hipMalloc(&staging, nbytes));
    HIP_CHECK(hipMemcpy(staging, bi.ptr, nbytes, hipMemcpyHostToDevice));
    if (qt == QT_F16 || qt == QT_BF16) HIP_CHECK(hipMemcpy(buf, staging, nbytes, hipMemcpyDeviceToDevice));
    else launch_repack(qt, staging, nb, w, nullptr);
    HIP_CHECK(hipDeviceSynchronize());
    HIP_CHECK(hipFree(staging));
  }
  ~PyQMatrix() {
    if (buf) hipFree(buf);
  }
};

}  // namespace

PYBIND11_MODULE(_engine, m) {
  m.doc() = "aiOS-MI355X native inference engine (gfx950 HIP kernels + C++ runtime)";
  m.attr("QT_F32") = (int)QT_F32;
  m.attr("QT_F16") = (int)QT_F16;
  m.attr("QT_BF16") = (int)QT_BF16;
  m.attr("QT_Q4_0") = (int)QT_Q4_0;
  m.attr("QT_Q8_0") = (int)QT_Q8_0;
  m.attr("QT_Q4_K") = (int)QT_Q4_K;
  m.attr("QT_Q5_K") = (int)QT_Q5_K;
  m.attr("QT_Q6_K") = (int)QT_Q6_K;
  m.attr("EPI_STORE") = (int)EPI_STORE;
  m.attr("EPI_RESID") = (int)EPI_RESID;
  m.attr("EPI_SWIGLU") = (int)EPI_SWIGLU;
  m.attr("EPI_QKV") = (int)EPI_QKV;
  m.attr("KV_BLOCK") = KV_BLOCK;
  m.attr("ATTN_CHUNK") = (int)ATTN_CHUNK;

  m.def("device_count", []() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
  });
  m.def("device_name", [](int dev) {
    hipDeviceProp_t p;
    HIP_CHECK(hipGetDeviceProperties(&p, dev));
    return std::string(p.name) + " / " + p.gcnArchName;
  });
  m.def("synchronize", []() { HIP_CHECK(hipDeviceSynchronize()); });
  m.def("resid_norm_parts", &resid_norm_parts, py::arg("d"));

  py::class_<EngineConfig>(m, "EngineConfig")
      .def(py::init<>())
      .def_readwrite("name", &EngineConfig::name)
      .def_readwrite("vocab_size", &EngineConfig::vocab_size)
      .def_readwrite("d_model", &EngineConfig::d_model)
      .def_readwrite("n_layers", &EngineConfig::n_layers)
      .def_readwrite("n_heads", &EngineConfig::n_heads)
      .def_readwrite("n_kv_heads", &EngineConfig::n_kv_heads)
      .def_readwrite("head_dim", &EngineConfig::head_dim)
      .def_readwrite("d_ff", &EngineConfig::d_ff)
      .def_readwrite("rope_theta", &EngineConfig::rope_theta)
      .def_readwrite("rope_neox", &EngineConfig::rope_neox)
      .def_readwrite("norm_eps", &EngineConfig::norm_eps)
      .def_readwrite("max_ctx", &EngineConfig::max_ctx)
      .def_readwrite("max_slots", &EngineConfig::max_slots)
      .def_readwrite("max_batch", &EngineConfig::max_batch)
      .def_readwrite("tie_embeddings", &EngineConfig::tie_embeddings)
      .def_readwrite("qk_norm", &EngineConfig::qk_norm)
      .def_readwrite("qkv_bias", &EngineConfig::qkv_bias)
      .def_readwrite("act_q8", &EngineConfig::act_q8)
      .def_readwrite("tp_rank", &EngineConfig::tp_rank)
      .def_readwrite("tp_size", &EngineConfig::tp_size)
      .def_readwrite("vocab_parallel", &EngineConfig::vocab_parallel)
      .def_readwrite("device", &EngineConfig::device)
      .def_readwrite("cu_mask", &EngineConfig::cu_mask)
      .def_readwrite("kv_fp8", &EngineConfig::kv_fp8)
      .def_readwrite("stream_priority", &EngineConfig::stream_priority);

  py::class_<Engine>(m, "Engine")
      .def(py::init<const EngineConfig&>())
      .def("set_tensor",
           [](Engine& e, const std::string& name, int qt, int rows, int cols, py::buffer raw) {
             py::buffer_info bi = raw.request();
             const size_t nbytes = (size_t)bi.size * bi.itemsize;
             py::gil_scoped_release nogil;
             e.set_tensor(name, qt, rows, cols, bi.ptr, nbytes);
           })
      .def("init_random", &Engine::init_random, py::call_guard<py::gil_scoped_release>())
      .def("finalize", &Engine::finalize, py::call_guard<py::gil_scoped_release>())
      .def("missing_tensors", &Engine::missing_tensors)
      .def("weight_type_summary", &Engine::weight_type_summary)
      .def_property_readonly("ready", &Engine::ready)
      .def_property_readonly("weight_bytes", &Engine::weight_bytes)
      .def_property_readonly("kv_bytes", &Engine::kv_bytes)
      .def_property_readonly("workspace_bytes", &Engine::workspace_bytes)
      .def_property_readonly("config", &Engine::config)
      .def("prefill",
           [](Engine& e, int slot, const std::vector<int>& tokens, int start_pos, bool want_logits) {
             std::vector<float> out;
             {
               py::gil_scoped_release nogil;
               out = e.prefill(slot, tokens, start_pos, want_logits);
             }
             return py::array_t<float>(out.size(), out.data());
           },
           py::arg("slot"), py::arg("tokens"), py::arg("start_pos") = 0, py::arg("want_logits") = true)
      .def("decode",
           [](Engine& e, const std::vector<int>& slots, const std::vector<int>& tokens, const std::vector<int>& pos,
              const std::vector<float>& temperature, const std::vector<int>& top_k, uint64_t seed, py::bytes mask,
              const std::vector<float>& top_p, const std::vector<uint64_t>& seeds) {
             std::string m = mask;  // packed allowed-token bitmask, B rows of ceil(V/8) bytes (or empty)
             std::vector<uint8_t> mv(m.begin(), m.end());
             py::gil_scoped_release nogil;
             return e.decode(slots, tokens, pos, temperature, top_k, seed, mv, top_p, seeds);
           },
           py::arg("slots"), py::arg("tokens"), py::arg("pos"), py::arg("temperature") = std::vector<float>{},
           py::arg("top_k") = std::vector<int>{}, py::arg("seed") = 0, py::arg("mask") = py::bytes(),
           py::arg("top_p") = std::vector<float>{}, py::arg("seeds") = std::vector<uint64_t>{})
      .def("decode_submit",
           [](Engine& e, const std::vector<int>& slots, const std::vector<int>& tokens, const std::vector<int>& pos,
              const std::vector<float>& temperature, const std::vector<int>& top_k, uint64_t seed,
              const std::vector<float>& top_p, const std::vector<uint64_t>& seeds) {
             py::gil_scoped_release nogil;
             e.decode_submit(slots, tokens, pos, temperature, top_k, seed, top_p, seeds);
           },
           py::arg("slots"), py::arg("tokens"), py::arg("pos"), py::arg("temperature") = std::vector<float>{},
           py::arg("top_k") = std::vector<int>{}, py::arg("seed") = 0, py::arg("top_p") = std::vector<float>{},
           py::arg("seeds") = std::vector<uint64_t>{})
      .def("decode_sample",
           [](Engine& e, py::bytes mask) {
             std::string m = mask;
             std::vector<uint8_t> mv(m.begin(), m.end());
             py::gil_scoped_release nogil;
             e.decode_sample(mv);
           },
           py::arg("mask") = py::bytes())
      .def("decode_collect", &Engine::decode_collect, py::call_guard<py::gil_scoped_release>())
      .def("sample_first",
           [](Engine& e, int pos, float temperature, int top_k, float top_p, uint64_t seed, py::bytes mask) {
             std::string m = mask;
             std::vector<uint8_t> mv(m.begin(), m.end());
             py::gil_scoped_release nogil;
             return e.sample_first(pos, temperature, top_k, top_p, seed, mv);
           },
           py::arg("pos"), py::arg("temperature") = 0.f, py::arg("top_k") = 0, py::arg("top_p") = 1.f,
           py::arg("seed") = 0, py::arg("mask") = py::bytes())
      .def("resample",
           [](Engine& e, int B, const std::vector<float>& temperature, const std::vector<int>& top_k, uint64_t seed,
              py::bytes mask, const std::vector<float>& top_p) {
             std::string m = mask;
             std::vector<uint8_t> mv(m.begin(), m.end());
             py::gil_scoped_release nogil;
             return e.resample(B, temperature, top_k, seed, mv, top_p);
           },
           py::arg("B"), py::arg("temperature") = std::vector<float>{}, py::arg("top_k") = std::vector<int>{},
           py::arg("seed") = 0, py::arg("mask") = py::bytes(), py::arg("top_p") = std::vector<float>{})
      .def("last_logits",
           [](Engine& e, int B) {
             std::vector<float> v;
             {
               py::gil_scoped_release nogil;
               v = e.last_logits(B);
             }
             py::array_t<float> a({(py::ssize_t)B, (py::ssize_t)e.config().vocab_size});
             std::memcpy(a.mutable_data(), v.data(), v.size() * 4);
             return a;
           })
      .def("decode_loop_prepare", &Engine::decode_loop_prepare, py::call_guard<py::gil_scoped_release>())
      .def("decode_loop_run", &Engine::decode_loop_run, py::arg("B"), py::arg("n_steps"), py::arg("use_graph") = true,
           py::call_guard<py::gil_scoped_release>())
      .def("decode_loop_history", &Engine::decode_loop_history, py::call_guard<py::gil_scoped_release>())
      .def("synchronize", &Engine::synchronize, py::call_guard<py::gil_scoped_release>())
      .def("reset_graphs", &Engine::reset_graphs)
      .def("copy_slot", &Engine::copy_slot, py::call_guard<py::gil_scoped_release>())
      .def("release_slot", &Engine::release_slot)
      .def("block_table", &Engine::block_table)
      .def_property_readonly("kv_blocks_free", &Engine::kv_blocks_free)
      .def_property_readonly("kv_blocks_total", &Engine::kv_blocks_total)
      .def_property_readonly("norm_fused_parts", &Engine::norm_fused_parts)
      .def("capture_graphs", &Engine::capture_graphs, py::arg("max_b"), py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("stream", &Engine::stream_handle)
      .def_property_readonly("k_cache_ptr", &Engine::kv_cache_k)
      .def_property_readonly("v_cache_ptr", &Engine::kv_cache_v)
      .def("set_allreduce_ptr", [](Engine& e, uintptr_t fn, uintptr_t ctx) {
        e.set_allreduce(reinterpret_cast<AllReduceFn>(fn), reinterpret_cast<void*>(ctx));
      })
      .def("set_comm", [](Engine& e, XgmiComm& c) {
        // the comm must outlive the engine's use of it (the Python wrapper keeps a reference)
        e.set_allreduce(&XgmiComm::hook, &c);
        e.set_allgather(&XgmiComm::gather_hook, &c);
        e.set_allreduce_norm(&XgmiComm::norm_hook, &c);
        e.set_tp_fuse(c.fuse_ctx(), c.fuse_grid());
      })
      .def("set_comm", [](Engine& e, RcclComm& c) {
        e.set_allreduce(&RcclComm::hook, &c);
        e.set_allgather(&RcclComm::gather_hook, &c);
        e.set_allreduce_norm(&RcclComm::norm_hook, &c);
      })
      .def_property_readonly("vocab_parallel", &Engine::vocab_parallel)
      .def_property_readonly("tp_fused", &Engine::tp_fused)
      .def("tp_fuse_fits", &Engine::tp_fuse_fits)
      .def("set_kv_scales", &Engine::set_kv_scales)
      .def_property_readonly("kv_scales", &Engine::kv_scales)
      .def_property_readonly("kv_fp8", &Engine::kv_fp8)
      .def("disable_tp_fuse", &Engine::disable_tp_fuse);

  // ------------------------------------------------------------------ TP collectives (xGMI)
  py::class_<XgmiComm>(m, "XgmiComm")
      .def(py::init<int, int, int, size_t>(), py::arg("rank"), py::arg("world"), py::arg("device"),
           py::arg("cap_floats"))
      .def("ipc_handle", [](const XgmiComm& c) { return py::bytes(c.ipc_handle()); })
      .def("set_ranks_per_gpu", &XgmiComm::set_ranks_per_gpu)
      .def_property_readonly("fuse_grid", &XgmiComm::fuse_grid)
      .def_property_readonly("fuse_eligible", &XgmiComm::fuse_eligible)
      .def_property_readonly("uncached", &XgmiComm::uncached)
      .def("disable_fuse", &XgmiComm::disable_fuse)
      .def_property_readonly("fused", [](const XgmiComm& c) { return c.fuse_ctx() != nullptr; })
      // one batch-1 EPI_TP_RESID GEMV through this comm's fused context (the TP init self-test of the
      // O / down all-reduce epilogue): y[n] += sum over ranks of (W x)[n]; false = not launched (no
      // fused context, or the shape does not fit the stage) -- dry: only whether it would launch
      .def("fused_gemv",
           [](XgmiComm& c, PyQMatrix& w, uintptr_t x, uintptr_t y, uintptr_t st, bool dry) {
             if (!c.fuse_ctx()) return false;
             GemvArgs a;
             std::memset(&a, 0, sizeof(a));
             a.nseg = 1; a.seg[0] = w.w; a.N = w.w.rows; a.K = w.w.cols; a.B = 1;
             a.x = (const float*)x; a.ldx = a.K; a.y = (float*)y; a.ldy = a.N;
             a.epi = EPI_TP_RESID; a.act_q8 = 1; a.tp = c.fuse_ctx(); a.kernel_sel = 1; a.grid_cap = c.fuse_grid();
             a.dry = dry ? 1 : 0;
             return launch_gemv_tp_fused(a, S(st));
           },
           py::arg("w"), py::arg("x"), py::arg("y"), py::arg("stream") = 0, py::arg("dry") = false)
      .def("connect", [](XgmiComm& c, const std::vector<py::bytes>& hs) {
        std::vector<std::string> v;
        for (auto& h : hs) v.push_back(std::string(h));
        c.connect(v);
      })
      .def("allreduce", [](XgmiComm& c, uintptr_t data, size_t n, uintptr_t residual, uintptr_t st) {
        c.allreduce((float*)data, n, (float*)residual, S(st));
      }, py::arg("data"), py::arg("n"), py::arg("residual") = 0, py::arg("stream") = 0)
      .def("allreduce_norm",
           [](XgmiComm& c, uintptr_t data, int rows, int d, uintptr_t residual, uintptr_t g, uintptr_t out16, int ld16,
              uintptr_t part, int parts, uintptr_t st) {
             c.allreduce_norm((float*)data, rows, d, (float*)residual,
                              ResidNorm{(const float*)g, (bf16_t*)out16, ld16, (float*)part, parts}, S(st));
           },
           py::arg("data"), py::arg("rows"), py::arg("d"), py::arg("residual"), py::arg("g"), py::arg("out16"),
           py::arg("ld16"), py::arg("part"), py::arg("parts"), py::arg("stream") = 0)
      .def("allgather_cols", [](XgmiComm& c, uintptr_t data, int rows, int slice, int ld, uintptr_t st) {
        c.allgather_cols((float*)data, rows, slice, ld, S(st));
      }, py::arg("data"), py::arg("rows"), py::arg("slice"), py::arg("ld"), py::arg("stream") = 0)
      .def_property("two_shot_min", &XgmiComm::two_shot_min, &XgmiComm::set_two_shot_min)
      .def_property("call_wg", &XgmiComm::call_wg, &XgmiComm::set_call_wg)
      .def_property("bf16_payload", &XgmiComm::bf16_payload, &XgmiComm::set_bf16_payload)
      .def("error", &XgmiComm::error)
      .def("reset_error", &XgmiComm::reset_error)
      .def_property_readonly("rank", &XgmiComm::rank)
      .def_property_readonly("world", &XgmiComm::world)
      .def_property_readonly("capacity", &XgmiComm::capacity)
      .def_property_readonly("connected", &XgmiComm::connected);

  // ------------------------------------------------------------------ TP collectives (RCCL, dlopen'd)
  py::class_<RcclComm>(m, "RcclComm")
      // the id arrives as std::string (converted under the GIL); only the collective init runs
      // without it (ncclCommInitRank blocks until every rank has joined)
      .def(py::init([](int rank, int world, int device, const std::string& id) {
             py::gil_scoped_release nogil;
             return new RcclComm(rank, world, device, id);
           }),
           py::arg("rank"), py::arg("world"), py::arg("device"), py::arg("unique_id"))
      .def_static("unique_id", []() { return py::bytes(RcclComm::unique_id()); })
      .def_static("available", &RcclComm::available)
      .def("allreduce", [](RcclComm& c, uintptr_t data, size_t n, uintptr_t residual, uintptr_t st) {
        c.allreduce((float*)data, n, (float*)residual, S(st));
      }, py::arg("data"), py::arg("n"), py::arg("residual") = 0, py::arg("stream") = 0)
      .def("allreduce_norm",
           [](RcclComm& c, uintptr_t data, int rows, int d, uintptr_t residual, uintptr_t g, uintptr_t out16, int ld16,
              uintptr_t part, int parts, uintptr_t st) {
             c.allreduce_norm((float*)data, rows, d, (float*)residual,
                              ResidNorm{(const float*)g, (bf16_t*)out16, ld16, (float*)part, parts}, S(st));
           },
           py::arg("data"), py::arg("rows"), py::arg("d"), py::arg("residual"), py::arg("g"), py::arg("out16"),
           py::arg("ld16"), py::arg("part"), py::arg("parts"), py::arg("stream") = 0)
      .def("allgather_cols", [](RcclComm& c, uintptr_t data, int rows, int slice, int ld, uintptr_t st) {
        c.allgather_cols((float*)data, rows, slice, ld, S(st));
      }, py::arg("data"), py::arg("rows"), py::arg("slice"), py::arg("ld"), py::arg("stream") = 0)
      .def("error", &RcclComm::error)
      .def("reset_error", &RcclComm::reset_error)
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("world", &RcclComm::world);

  // ------------------------------------------------------------------ raw ops (tests / tools)
  py::class_<PyQMatrix>(m, "QMatrix")
      .def(py::init<int, int, int, py::buffer>())
      .def_property_readonly("qtype", [](const PyQMatrix& q) { return q.w.qtype; })
      .def_property_readonly("rows", [](const PyQMatrix& q) { return q.w.rows; })
      .def_property_readonly("cols", [](const PyQMatrix& q) { return q.w.cols; })
      .def_property_readonly("nbytes", [](const PyQMatrix& q) { return q.bytes; })
      .def("dequant_bf16", [](PyQMatrix& q, uintptr_t out, uintptr_t st) { launch_dequant_bf16(q.w, (void*)out, S(st)); })
      .def("get_rows", [](PyQMatrix& q, uintptr_t rows, int n, uintptr_t out, int ldo, uintptr_t st) {
        launch_get_rows(q.w, (const int*)rows, n, (float*)out, ldo, 1.f, S(st));
      })
      .def("fill_random", [](PyQMatrix& q, uint64_t seed, float amp) {
        fill_random_weight(q.w, seed, amp, nullptr);
        HIP_CHECK(hipDeviceSynchronize());
      });

  m.def("gemv",
        [](std::vector<PyQMatrix*> segs, int B, uintptr_t x, int ldx, uintptr_t norm_w, float eps, uintptr_t y,
           int ldy, int epi, uintptr_t st, int force_v1, int act_q8, int tune_grid, int tune_u, int tune_ksplit, int tune_dbg,
           int kernel_sel, uintptr_t dbg_ts, uintptr_t x16, uintptr_t y16) {
          GemvArgs a;
          std::memset(&a, 0, sizeof(a));
          a.nseg = (int)segs.size();
          int r = 0;
          for (int s = 0; s < a.nseg; ++s) { a.seg[s] = segs[s]->w; a.seg_row0[s] = r; r += segs[s]->w.rows; }
          a.N = r; a.K = segs[0]->w.cols; a.B = B;
          a.x = (const float*)x; a.ldx = ldx; a.norm_w = (const float*)norm_w; a.eps = eps;
          a.y = (float*)y; a.ldy = ldy; a.epi = epi; a.force_v1 = force_v1; a.act_q8 = act_q8;
          a.tune_grid = tune_grid; a.tune_u = tune_u; a.tune_ksplit = tune_ksplit; a.tune_dbg = tune_dbg;
          a.kernel_sel = kernel_sel; a.dbg_ts = (unsigned long long*)dbg_ts;
          a.x16 = (const bf16_t*)x16; a.y16 = (bf16_t*)y16;  // bf16 input / SwiGLU output (hand-off kernels)
          launch_gemv(a, S(st));
        },
        py::arg("segs"), py::arg("B"), py::arg("x"), py::arg("ldx"), py::arg("norm_w"), py::arg("eps"), py::arg("y"),
        py::arg("ldy"), py::arg("epi"), py::arg("stream"), py::arg("force_v1") = 0, py::arg("act_q8") = 0,
        py::arg("tune_grid") = 0, py::arg("tune_u") = 0, py::arg("tune_ksplit") = 0, py::arg("tune_dbg") = 0,
        py::arg("kernel_sel") = 0, py::arg("dbg_ts") = 0, py::arg("x16") = 0, py::arg("y16") = 0);
  m.def("gemv_bf16_engine_fits",
        [](std::vector<PyQMatrix*> segs, int B, int epi) {
          GemvArgs a;
          std::memset(&a, 0, sizeof(a));
          a.nseg = (int)segs.size();
          int r = 0;
          for (int s = 0; s < a.nseg; ++s) { a.seg[s] = segs[s]->w; a.seg_row0[s] = r; r += segs[s]->w.rows; }
          a.N = r; a.K = segs[0]->w.cols; a.B = B; a.epi = epi;
          return gemv_bf16_engine_fits(a);
        },
        py::arg("segs"), py::arg("B"), py::arg("epi") = 0);
  m.def("gemv_qkv",
        [](std::vector<PyQMatrix*> segs, int B, uintptr_t x, int ldx, uintptr_t norm_w, float eps, uintptr_t q_out,
           uintptr_t bias, int head_dim, int n_heads, int n_kv_heads, int max_ctx, int rope_neox, float rope_base,
           uintptr_t pos, uintptr_t slot, uintptr_t k_cache, uintptr_t v_cache, uintptr_t st, int act_q8,
           uintptr_t block_table, uintptr_t rope_cs, int tune_grid, int kernel_sel) {
          GemvArgs a;
          std::memset(&a, 0, sizeof(a));
          a.nseg = (int)segs.size();
          int r = 0;
          for (int s = 0; s < a.nseg; ++s) { a.seg[s] = segs[s]->w; a.seg_row0[s] = r; r += segs[s]->w.rows; }
          a.N = r; a.K = segs[0]->w.cols; a.B = B;
          a.x = (const float*)x; a.ldx = ldx; a.norm_w = (const float*)norm_w; a.eps = eps;
          a.y = (float*)q_out; a.ldy = n_heads * head_dim; a.epi = EPI_QKV;
          a.bias = (const float*)bias; a.head_dim = head_dim; a.q_dim = n_heads * head_dim;
          a.kv_dim = n_kv_heads * head_dim; a.n_kv_heads = n_kv_heads; a.max_ctx = max_ctx;
          a.rope_neox = rope_neox; a.rope_base = rope_base; a.rope_cs = (const float2*)rope_cs; a.pos = (const int*)pos; a.slot = (const int*)slot;
          a.k_cache = (bf16_t*)k_cache; a.v_cache = (bf16_t*)v_cache; a.act_q8 = act_q8;
          a.block_table = (const int*)block_table;
          a.tune_grid = tune_grid;
          a.kernel_sel = kernel_sel;
          launch_gemv(a, S(st));
        },
        py::arg("segs"), py::arg("B"), py::arg("x"), py::arg("ldx"), py::arg("norm_w"), py::arg("eps"),
        py::arg("q_out"), py::arg("bias"), py::arg("head_dim"), py::arg("n_heads"), py::arg("n_kv_heads"),
        py::arg("max_ctx"), py::arg("rope_neox"), py::arg("rope_base"), py::arg("pos"), py::arg("slot"),
        py::arg("k_cache"), py::arg("v_cache"), py::arg("stream"), py::arg("act_q8") = 0,
        py::arg("block_table") = 0, py::arg("rope_cs") = 0, py::arg("tune_grid") = 0, py::arg("kernel_sel") = 0);
  m.def("attn_decode",
        [](uintptr_t q, uintptr_t k, uintptr_t v, uintptr_t seq_len, uintptr_t slot, int B, int H, int Hkv, int hd,
           int max_ctx, int n_chunks, float scale, uintptr_t opart, uintptr_t ml, uintptr_t out, uintptr_t counters,
           uintptr_t st, int split, uintptr_t block_table, int bt_rows, uintptr_t ts, int kv_fp8, float k_scale,
           float v_scale) {
          AttnDecodeArgs a;
          a.split = split;
          a.kv_fp8 = kv_fp8; a.kv_scale_k = k_scale; a.kv_scale_v = v_scale;
          a.ts = (unsigned long long*)ts;
          a.block_table = (const int*)block_table; a.bt_rows = bt_rows;
          a.q = (const float*)q; a.k_cache = (const bf16_t*)k; a.v_cache = (const bf16_t*)v;
          a.seq_len = (const int*)seq_len; a.slot = (const int*)slot;
          a.B = B; a.n_heads = H; a.n_kv_heads = Hkv; a.head_dim = hd; a.max_ctx = max_ctx; a.n_chunks = n_chunks;
          a.scale = scale; a.o_part = (float*)opart; a.ml = (float*)ml; a.out = (float*)out;
          a.counters = (int*)counters;
          launch_attn_decode(a, S(st));
        },
        py::arg("q"), py::arg("k"), py::arg("v"), py::arg("seq_len"), py::arg("slot"), py::arg("B"), py::arg("H"),
        py::arg("Hkv"), py::arg("hd"), py::arg("max_ctx"), py::arg("n_chunks"), py::arg("scale"), py::arg("opart"),
        py::arg("ml"), py::arg("out"), py::arg("counters"), py::arg("st"), py::arg("split") = 0,
        py::arg("block_table") = 0, py::arg("bt_rows") = 0, py::arg("ts") = 0, py::arg("kv_fp8") = 0,
        py::arg("k_scale") = 1.f, py::arg("v_scale") = 1.f);
  m.def("attn_decode_split", &attn_decode_split);
  // physical identity of a device (PCI bus id): ranks that share a GPU see the same string
  m.def("device_cu_count", [](int dev) {
    int n = 0;
    HIP_CHECK(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
    return n;
  }, py::arg("device") = 0);
  m.def("device_pci_bus_id", [](int dev) {
    char buf[64] = {0};
    HIP_CHECK(hipDeviceGetPCIBusId(buf, (int)sizeof(buf), dev));
    return std::string(buf);
  });
  m.def("rmsnorm", [](uintptr_t x, int ldx, uintptr_t w, uintptr_t y, int ldy, int rows, int n, float eps, uintptr_t st) {
    launch_rmsnorm((const float*)x, ldx, (const float*)w, (float*)y, ldy, rows, n, eps, S(st));
  });
  m.def("rmsnorm_bf16", [](uintptr_t x, int ldx, uintptr_t w, uintptr_t y, int ldy, int rows, int n, float eps, uintptr_t st) {
    launch_rmsnorm_bf16((const float*)x, ldx, (const float*)w, (bf16_t*)y, ldy, rows, n, eps, S(st));
  });
  m.def("swiglu", [](uintptr_t gu, int ldg, uintptr_t out, int ldo, int rows, int n, uintptr_t st) {
    launch_swiglu_interleaved((const float*)gu, ldg, (float*)out, ldo, rows, n, S(st));
  });
  m.def("qkv_post",
        [](uintptr_t qkv, int ldqkv, int T, int H, int Hkv, int hd, uintptr_t q_norm, uintptr_t k_norm, float eps,
           int rope_neox, float rope_base, uintptr_t pos, uintptr_t slot, uintptr_t q_out, uintptr_t k_cache,
           uintptr_t v_cache, int max_ctx, uintptr_t st, uintptr_t block_table) {
          QkvPostArgs a;
          a.block_table = (const int*)block_table;
          a.qkv = (const float*)qkv; a.ldqkv = ldqkv; a.T = T; a.n_heads = H; a.n_kv_heads = Hkv; a.head_dim = hd;
          a.q_norm = (const float*)q_norm; a.k_norm = (const float*)k_norm; a.eps = eps; a.rope_neox = rope_neox;
          a.rope_base = rope_base; a.rope_cs = nullptr; a.pos = (const int*)pos; a.slot = (const int*)slot; a.q_out = (float*)q_out;
          a.k_cache = (bf16_t*)k_cache; a.v_cache = (bf16_t*)v_cache; a.max_ctx = max_ctx;
          launch_qkv_post(a, S(st));
        },
        py::arg("qkv"), py::arg("ldqkv"), py::arg("T"), py::arg("H"), py::arg("Hkv"), py::arg("hd"), py::arg("q_norm"),
        py::arg("k_norm"), py::arg("eps"), py::arg("rope_neox"), py::arg("rope_base"), py::arg("pos"), py::arg("slot"),
        py::arg("q_out"), py::arg("k_cache"), py::arg("v_cache"), py::arg("max_ctx"), py::arg("st"),
        py::arg("block_table") = 0);
  m.def("sample",
        [](uintptr_t logits, int ldl, int B, int V, uintptr_t temperature, uintptr_t top_k, uint64_t seed,
           uintptr_t tokens, uintptr_t pos, uintptr_t mask, uintptr_t st, uintptr_t top_p, uintptr_t ts) {
          // grow-on-demand scratch for the raw-op binding (the engine owns its own)
          static void* ws = nullptr;
          static size_t ws_bytes = 0;
          static int* cnt = nullptr;
          static int cnt_len = 0;
          const size_t need = sample_ws_bytes(B, V);
          if (need > ws_bytes) {
            if (ws) HIP_CHECK(hipFree(ws));
            HIP_CHECK(hipMalloc(&ws, need));
            ws_bytes = need;
          }
          if (B > cnt_len) {
            if (cnt) HIP_CHECK(hipFree(cnt));
            HIP_CHECK(hipMalloc(&cnt, (size_t)B * 4));
            HIP_CHECK(hipMemset(cnt, 0, (size_t)B * 4));
            cnt_len = B;
          }
          SampleArgs a;
          std::memset(&a, 0, sizeof(a));
          a.logits = (const float*)logits; a.ldl = ldl; a.B = B; a.V = V;
          a.temperature = (const float*)temperature; a.top_k = (const int*)top_k; a.seed = seed;
          a.tokens = (int*)tokens; a.pos = (int*)pos; a.mask = (const uint8_t*)mask;
          a.top_p = (const float*)top_p; a.ws = ws; a.ws_bytes = ws_bytes; a.counters = cnt;
          a.ts = (long long*)ts;
          launch_sample(a, S(st));
        },
        py::arg("logits"), py::arg("ldl"), py::arg("B"), py::arg("V"), py::arg("temperature"), py::arg("top_k"),
        py::arg("seed"), py::arg("tokens"), py::arg("pos"), py::arg("mask"), py::arg("st"), py::arg("top_p") = 0,
        py::arg("ts") = 0);
  m.def("gemm",
        [](uintptr_t A, int lda, PyQMatrix* w, int M, uintptr_t C, int ldc, int accumulate, uintptr_t st) {
          GemmArgs a;
          a.A = (const bf16_t*)A; a.lda = lda; a.w = w->w; a.M = M; a.N = w->w.rows; a.K = w->w.cols;
          a.C = (float*)C; a.ldc = ldc; a.accumulate = accumulate;
          GemmWs& g = gemm_ws(M, a.N);
          a.ws = g.ws; a.ws_bytes = g.bytes; a.cnt = g.cnt; a.cnt_len = g.cnt_len;
          launch_gemm(a, S(st));
        });
  m.def("gemm_supports", &gemm_supports);
  m.def(
      "gemm_q",
      [](uintptr_t A, int lda, std::vector<PyQMatrix*> segs, int M, uintptr_t C, uintptr_t C16, int ldc, int epi,
         uintptr_t st, int ksplit, uintptr_t dbg_ts) {
        GemmQArgs a;
        std::memset(&a, 0, sizeof(a));
        if (segs.empty() || segs.size() > 3) throw std::runtime_error("gemm_q: 1..3 segments");
        a.A = (const bf16_t*)A; a.lda = lda; a.nseg = (int)segs.size();
        int n0 = 0;
        for (int s = 0; s < a.nseg; ++s) { a.seg[s] = segs[s]->w; a.seg_n0[s] = n0; n0 += segs[s]->w.rows; }
        a.M = M; a.N = n0; a.K = segs[0]->w.cols;
        a.C = (float*)C; a.C16 = (bf16_t*)C16; a.ldc = ldc; a.epi = epi; a.ksplit = ksplit;
        a.dbg_ts = (unsigned long long*)dbg_ts;
        GemmWs& g = gemm_ws(M, a.N);
        a.ws = g.ws; a.ws_bytes = g.bytes; a.cnt = g.cnt; a.cnt_len = g.cnt_len;
        launch_gemm_q(a, S(st));
      },
      py::arg("A"), py::arg("lda"), py::arg("segs"), py::arg("M"), py::arg("C"), py::arg("C16"), py::arg("ldc"),
      py::arg("epi"), py::arg("stream"), py::arg("ksplit") = 0, py::arg("dbg_ts") = 0);
  m.def(
      "gemm_pf_plan",
      [](std::vector<PyQMatrix*> segs, int M, int epi, int ksplit) {
        GemmQArgs a;
        std::memset(&a, 0, sizeof(a));
        if (segs.empty() || segs.size() > 3) throw std::runtime_error("gemm_pf_plan: 1..3 segments");
        a.nseg = (int)segs.size();
        int n0 = 0;
        for (int s = 0; s < a.nseg; ++s) { a.seg[s] = segs[s]->w; a.seg_n0[s] = n0; n0 += segs[s]->w.rows; }
        a.M = M; a.N = n0; a.K = segs[0]->w.cols; a.epi = epi; a.ksplit = ksplit;
        int bm = 0, bn = 0, sp = 0;
        gemm_pf_plan(a, bm, bn, sp);
        return py::make_tuple(bm, bn, sp);
      },
      py::arg("segs"), py::arg("M"), py::arg("epi"), py::arg("ksplit") = 0);
  m.def(
      "gemm_pf_probe",
      [](uintptr_t A, int lda, PyQMatrix* w, int M, uintptr_t C, int probe, uintptr_t st) {
        GemmQArgs a;
        std::memset(&a, 0, sizeof(a));
        a.A = (const bf16_t*)A; a.lda = lda; a.nseg = 1; a.seg[0] = w->w; a.M = M; a.N = w->w.rows;
        a.K = w->w.cols; a.C = (float*)C; a.ldc = a.N; a.epi = GEPI_STORE;
        return gemm_pf_probe(a, probe, S(st));
      });
  m.attr("GEPI_STORE") = (int)GEPI_STORE;
  m.attr("GEPI_ACCUM") = (int)GEPI_ACCUM;
  m.attr("GEPI_SWIGLU_BF16") = (int)GEPI_SWIGLU_BF16;
  m.def(
      "attn_prefill",
      [](uintptr_t q, uintptr_t k, uintptr_t v, int slot, int start, int T, int H, int Hkv, int hd, int max_ctx,
         float scale, uintptr_t out, int ldo, uintptr_t st, uintptr_t block_table, int kv_fp8, float k_scale,
         float v_scale) {
        AttnPrefillArgs a;
        a.kv_fp8 = kv_fp8; a.kv_scale_k = k_scale; a.kv_scale_v = v_scale;
        a.block_table = (const int*)block_table;
        a.q = (const float*)q; a.k_cache = (const bf16_t*)k; a.v_cache = (const bf16_t*)v;
        a.slot = slot; a.start = start; a.T = T; a.n_heads = H; a.n_kv_heads = Hkv; a.head_dim = hd;
        a.max_ctx = max_ctx; a.scale = scale; a.out = (bf16_t*)out; a.ldo = ldo;
        launch_attn_prefill(a, S(st));
      },
      py::arg("q"), py::arg("k"), py::arg("v"), py::arg("slot"), py::arg("start"), py::arg("T"), py::arg("H"),
      py::arg("Hkv"), py::arg("hd"), py::arg("max_ctx"), py::arg("scale"), py::arg("out"), py::arg("ldo"),
      py::arg("st"), py::arg("block_table") = 0, py::arg("kv_fp8") = 0, py::arg("k_scale") = 1.f,
      py::arg("v_scale") = 1.f);
  m.def("attn_prefill_supports", &attn_prefill_supports);

  // ------------------------------------------------------------------ JSON-mode grammar (K10)
  py::class_<JsonState>(m, "JsonState")
      .def(py::init<>())
      .def("copy", [](const JsonState& s) { return JsonState(s); })
      .def_property_readonly("depth", [](const JsonState& s) { return (int)s.depth; })
      .def_property_readonly("mode", [](const JsonState& s) { return (int)s.mode; });
  py::class_<JsonGrammar>(m, "JsonGrammar")
      .def(py::init([](const std::vector<py::bytes>& toks, int eos, int max_ws, bool require_object) {
             std::vector<std::string> t;
             t.reserve(toks.size());
             for (auto& b : toks) t.push_back(std::string(b));
             return new JsonGrammar(t, eos, max_ws, require_object);
           }),
           py::arg("tokens"), py::arg("eos_id"), py::arg("max_ws") = 20, py::arg("require_object") = true)
      .def("initial", &JsonGrammar::initial)
      .def("accept_token", &JsonGrammar::accept_token)
      .def("accept_bytes", [](const JsonGrammar& g, JsonState& s, py::bytes b) { return g.accept_bytes(s, std::string(b)); })
      .def("complete", &JsonGrammar::complete)
      .def("mask",
           [](JsonGrammar& g, const JsonState& s) {
             const std::vector<uint8_t>* m;
             {
               py::gil_scoped_release nogil;
               m = &g.mask(s);
             }
             return py::bytes((const char*)m->data(), m->size());
           })
      .def("mask_open",
           [](JsonGrammar& g, const JsonState& s) {
             const std::vector<uint8_t>* m;
             {
               py::gil_scoped_release nogil;
               m = &g.mask_open(s);
             }
             return py::bytes((const char*)m->data(), m->size());
           })
      .def_property_readonly("vocab_size", &JsonGrammar::vocab_size)
      .def_property_readonly("cache_size", &JsonGrammar::cache_size);
  m.def("gemm_pf_export", &gemm_pf_export);
  m.def("gemm_pf_import", &gemm_pf_import, py::arg("plans"));
  m.def("bench_stream_read_part", &aios::bench_stream_read_part, py::arg("bytes"), py::arg("nbuf"), py::arg("mode"),
        py::arg("threads") = 512, py::arg("reps") = 20);
  m.def("bench_stream_read", &aios::bench_stream_read, py::arg("bytes"), py::arg("nbuf"), py::arg("wg_per_cu"),
        py::arg("u"), py::arg("threads"), py::arg("reps"));
  m.def("bench_launch_chain", &aios::bench_launch_chain, py::arg("n_kernels"), py::arg("blocks"), py::arg("use_graph"),
        py::arg("reps"), py::call_guard<py::gil_scoped_release>());
}
