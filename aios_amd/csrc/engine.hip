// Engine implementation -- see engine.h.
#include "engine.h"
#include <hip/hip_ext.h>

#include <set>
#include "comm.h"
#include <cstdlib>
#include <map>

#include <algorithm>
#include <cstring>
#include <cmath>
#include <regex>
#include <sstream>

#include <rocprofiler-sdk-roctx/roctx.h>

namespace aios {

static bool trace_enabled() {
  static const int on = [] {
    const char* e = std::getenv("AIOS_TRACE");
    return e && std::atoi(e) == 0 ? 0 : 1;
  }();
  return on != 0;
}
TraceRange::TraceRange(const char* name) : on(trace_enabled()) {
  if (on) roctxRangePushA(name);
}
TraceRange::~TraceRange() {
  if (on) roctxRangePop();
}

static size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

static bool is_kquant(int qt) { return qt == QT_Q4_K || qt == QT_Q5_K || qt == QT_Q6_K; }
static int block_elems(int qt) {
  if (is_kquant(qt) || qt == QT_Q2_K || qt == QT_Q3_K || qt == QT_IQ4_XS) return 256;
  if (qt == QT_F32 || qt == QT_F16 || qt == QT_BF16) return 1;
  return 32;
}
static int block_bytes(int qt) {
  switch (qt) {
    case QT_Q4_K: return 144;
    case QT_Q5_K: return 176;
    case QT_Q6_K: return 210;
    case QT_Q4_0: return 18;
    case QT_Q4_1: return 20;
    case QT_Q5_0: return 22;
    case QT_Q5_1: return 24;
    case QT_Q8_0: return 34;
    case QT_Q2_K: return 84;
    case QT_Q3_K: return 110;
    case QT_IQ4_NL: return 18;
    case QT_IQ4_XS: return 136;
    case QT_F16:
    case QT_BF16: return 2;
    case QT_F32: return 4;
  }
  throw std::runtime_error("unsupported ggml type " + std::to_string(qt));
}
// formats the GEMV streams natively; others are expanded to BF16 at load
static bool native_qtype(int qt) {
  return qt == QT_Q4_K || qt == QT_Q5_K || qt == QT_Q6_K || qt == QT_Q4_0 || qt == QT_Q8_0 || qt == QT_F16 ||
         qt == QT_BF16;
}

Engine::Engine(const EngineConfig& cfg) : cfg_(cfg) {
  HIP_CHECK(hipSetDevice(cfg_.device));
  if (!cfg_.cu_mask.empty()) {
    int n = 0, dev_cus = 0;
    for (uint32_t w : cfg_.cu_mask) n += __builtin_popcount(w);
    HIP_CHECK(hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, cfg_.device));
    if (n <= 0) throw std::runtime_error("cu_mask selects no CU");
    HIP_CHECK(hipExtStreamCreateWithCUMask(&stream_, (uint32_t)cfg_.cu_mask.size(), cfg_.cu_mask.data()));
    cus_ = std::min(n, dev_cus);
  } else if (cfg_.stream_priority != 0) {
    int least = 0, greatest = 0;
    HIP_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    const int pr = std::max(greatest, std::min(least, cfg_.stream_priority));
    HIP_CHECK(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, pr));
  } else {
    HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  }

  layers_.resize(cfg_.n_layers);
  // B <= 8 decodes through the fused GEMVs; larger batches (up to 64) through the MFMA GEMM path
  if (cfg_.max_batch < 1 || cfg_.max_batch > 64) throw std::runtime_error("max_batch must be 1..64");
  if (cfg_.max_slots < cfg_.max_batch) cfg_.max_slots = cfg_.max_batch;
  if (cfg_.tp_size <= 1 || cfg_.tie_embeddings) cfg_.vocab_parallel = 0;
  if (cfg_.vocab_parallel && cfg_.vocab_size % cfg_.tp_size)
    throw std::runtime_error("vocab_parallel: vocab_size not divisible by tp_size");
}

Engine::~Engine() {
  try {
    stage_release();
  } catch (...) {
  }
  for (auto& kv : graphs_) hipGraphExecDestroy(kv.second);
  for (void* p : allocs_) hipFree(p);
  if (h_par_) hipHostFree(h_par_);
  if (h_tok_out_) hipHostFree(h_tok_out_);
  if (h_mask_) hipHostFree(h_mask_);
  if (pipe_ev_) hipEventDestroy(pipe_ev_);
  if (stream_) hipStreamDestroy(stream_);
}

void* Engine::dmalloc(size_t bytes) {
  void* p = nullptr;
  HIP_CHECK(hipMalloc(&p, std::max<size_t>(bytes, 16)));
  allocs_.push_back(p);
  return p;
}

QMat Engine::alloc_qmat(int qt, int rows, int cols) {
  if (cols % block_elems(qt)) throw std::runtime_error("matrix cols not a multiple of the quant block");
  QMat m;
  m.w.qtype = qt;
  m.w.rows = rows;
  m.w.cols = cols;
  const size_t nb = (size_t)rows * (cols / block_elems(qt));
  size_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
  switch (qt) {
    case QT_Q4_K: s0 = nb * 128; s1 = nb * 16; break;
    case QT_Q5_K: s0 = nb * 128; s1 = nb * 16; s2 = nb * 32; break;
    case QT_Q6_K: s0 = nb * 128; s1 = nb * 64; s2 = nb * 16; s3 = nb * 2; break;
    case QT_Q4_0: s0 = nb * 16; s1 = nb * 2; break;
    case QT_Q8_0: s0 = nb * 32; s1 = nb * 2; break;
    case QT_F16:
    case QT_BF16: s0 = (size_t)rows * cols * 2; break;
    default: throw std::runtime_error("alloc_qmat: non-native type");
  }
  const size_t a = 256;
  const size_t o1 = align_up(s0, a), o2 = o1 + align_up(s1, a), o3 = o2 + align_up(s2, a);
  m.bytes = o3 + align_up(s3, a) + 64;
  m.buf = dmalloc(m.bytes);
  uint8_t* base = (uint8_t*)m.buf;
  m.w.p0 = base;
  m.w.p1 = s1 ? base + o1 : nullptr;
  m.w.p2 = s2 ? base + o2 : nullptr;
  m.w.p3 = s3 ? base + o3 : nullptr;
  weight_bytes_ += m.bytes;
  return m;
}

// Load path (one hipMalloc + pageable copy + stream sync + hipFree per tensor).
// Now: the GGUF bytes (mmap'd by the loader) are copied in 64 MB chunks through two pinned host
// buffers into one of two device staging buffers (DMA from pinned memory, the next chunk's host
// memcpy overlapping the previous chunk's transfer), and the repack kernel of tensor i runs while
// tensor i+1 is being staged into the other buffer.  No per-tensor allocation or device sync.
void Engine::stage_upload(const void* host, size_t nbytes, void*& dev_staging) {
  constexpr size_t CHUNK = 64ull << 20;
  const int k = stage_next_;
  stage_next_ ^= 1;
  if (stage_ev_[k]) HIP_CHECK(hipEventSynchronize(stage_ev_[k]));  // repack of the tensor two back is done
  if (stage_dev_bytes_[k] < nbytes) {
    if (stage_dev_[k]) HIP_CHECK(hipFree(stage_dev_[k]));
    stage_dev_bytes_[k] = std::max(nbytes, (size_t)256 << 20);
    HIP_CHECK(hipMalloc(&stage_dev_[k], stage_dev_bytes_[k]));
  }
  for (int i = 0; i < 2; ++i)
    if (!stage_host_[i]) {
      HIP_CHECK(hipHostMalloc(&stage_host_[i], CHUNK, hipHostMallocDefault));
      HIP_CHECK(hipEventCreateWithFlags(&stage_host_ev_[i], hipEventDisableTiming));
      HIP_CHECK(hipEventRecord(stage_host_ev_[i], stream_));
    }
  for (size_t off = 0; off < nbytes; off += CHUNK) {
    const size_t n = std::min(CHUNK, nbytes - off);
    const int h = stage_host_next_;
    stage_host_next_ ^= 1;
    HIP_CHECK(hipEventSynchronize(stage_host_ev_[h]));  // this pinned buffer's last transfer is done
    std::memcpy(stage_host_[h], (const uint8_t*)host + off, n);
    HIP_CHECK(hipMemcpyAsync((uint8_t*)stage_dev_[k] + off, stage_host_[h], n, hipMemcpyHostToDevice, stream_));
    HIP_CHECK(hipEventRecord(stage_host_ev_[h], stream_));
  }
  dev_staging = stage_dev_[k];
  stage_cur_ = k;
}

void Engine::stage_done() {
  const int k = stage_cur_;
  if (!stage_ev_[k]) HIP_CHECK(hipEventCreateWithFlags(&stage_ev_[k], hipEventDisableTiming));
  HIP_CHECK(hipEventRecord(stage_ev_[k], stream_));
}

void Engine::stage_release() {
  HIP_CHECK(hipStreamSynchronize(stream_));
  for (int i = 0; i < 2; ++i) {
    if (stage_dev_[i]) HIP_CHECK(hipFree(stage_dev_[i]));
    if (stage_host_[i]) HIP_CHECK(hipHostFree(stage_host_[i]));
    if (stage_ev_[i]) HIP_CHECK(hipEventDestroy(stage_ev_[i]));
    if (stage_host_ev_[i]) HIP_CHECK(hipEventDestroy(stage_host_ev_[i]));
    stage_dev_[i] = stage_host_[i] = nullptr;
    stage_ev_[i] = stage_host_ev_[i] = nullptr;
    stage_dev_bytes_[i] = 0;
  }
}

QMat Engine::upload_qmat(int qt, int rows, int cols, const void* host, size_t nbytes) {
  const size_t expect = (size_t)rows * (cols / block_elems(qt)) * block_bytes(qt);
  if (nbytes != expect)
    throw std::runtime_error("tensor byte size mismatch: got " + std::to_string(nbytes) + " expected " +
                             std::to_string(expect));
  QMat m;
  if ((qt == QT_F16 || qt == QT_BF16)) {  // final layout == file layout: straight into place
    m = alloc_qmat(qt, rows, cols);
    void* staging = nullptr;
    stage_upload(host, nbytes, staging);
    HIP_CHECK(hipMemcpyAsync(m.buf, staging, nbytes, hipMemcpyDeviceToDevice, stream_));
    stage_done();
    return m;
  }
  void* staging = nullptr;
  stage_upload(host, nbytes, staging);
  if (native_qtype(qt)) {
    m = alloc_qmat(qt, rows, cols);
    launch_repack(qt, staging, (size_t)rows * (cols / block_elems(qt)), m.w, stream_);
  } else {
    m = alloc_qmat(QT_BF16, rows, cols);
    launch_legacy_to_bf16(qt, staging, (size_t)rows * cols, m.buf, stream_);
  }
  stage_done();
  return m;
}

float* Engine::upload_f32(const void* host, size_t n, int qt) {
  std::vector<float> tmp(n);
  if (qt == QT_F32) {
    std::memcpy(tmp.data(), host, n * 4);
  } else if (qt == QT_F16 || qt == QT_BF16) {
    const uint16_t* h = (const uint16_t*)host;
    for (size_t i = 0; i < n; ++i) {
      if (qt == QT_BF16) {
        uint32_t u = (uint32_t)h[i] << 16;
        std::memcpy(&tmp[i], &u, 4);
      } else {
        // IEEE half -> float
        const uint32_t s = (h[i] >> 15) & 1, e = (h[i] >> 10) & 31, f = h[i] & 1023;
        float v;
        if (e == 0) v = std::ldexp((float)f, -24);
        else if (e == 31) v = f ? NAN : INFINITY;
        else v = std::ldexp((float)(f | 1024), (int)e - 25);
        tmp[i] = s ? -v : v;
      }
    }
  } else {
    throw std::runtime_error("norm/bias tensors must be F32/F16/BF16");
  }
  float* d = (float*)dmalloc(n * 4);
  HIP_CHECK(hipMemcpy(d, tmp.data(), n * 4, hipMemcpyHostToDevice));
  weight_bytes_ += n * 4;
  return d;
}

// rows of a and b interleaved: out row 2i = a row i, 2i+1 = b row i (gate/up -> SwiGLU pairs)
QMat Engine::interleave_rows(const QMat& a, const QMat& b) {
  if (a.w.qtype != b.w.qtype || a.w.rows != b.w.rows || a.w.cols != b.w.cols)
    throw std::runtime_error("gate/up shape or format mismatch");
  QMat m = alloc_qmat(a.w.qtype, 2 * a.w.rows, a.w.cols);
  const int rows = a.w.rows;
  const size_t nbr = a.w.cols / block_elems(a.w.qtype);  // blocks per row
  auto copy_stream = [&](const uint8_t* dst, const uint8_t* sa, const uint8_t* sb, size_t row_bytes) {
    if (!dst) return;
    HIP_CHECK(hipMemcpy2DAsync((void*)dst, 2 * row_bytes, sa, row_bytes, row_bytes, rows, hipMemcpyDeviceToDevice,
                               stream_));
    HIP_CHECK(hipMemcpy2DAsync((void*)(dst + row_bytes), 2 * row_bytes, sb, row_bytes, row_bytes, rows,
                               hipMemcpyDeviceToDevice, stream_));
  };
  size_t r0 = 0, r1 = 0, r2 = 0, r3 = 0;
  switch (a.w.qtype) {
    case QT_Q4_K: r0 = nbr * 128; r1 = nbr * 16; break;
    case QT_Q5_K: r0 = nbr * 128; r1 = nbr * 16; r2 = nbr * 32; break;
    case QT_Q6_K: r0 = nbr * 128; r1 = nbr * 64; r2 = nbr * 16; r3 = nbr * 2; break;
    case QT_Q4_0: r0 = nbr * 16; r1 = nbr * 2; break;
    case QT_Q8_0: r0 = nbr * 32; r1 = nbr * 2; break;
    default: r0 = (size_t)a.w.cols * 2; break;
  }
  copy_stream(m.w.p0, a.w.p0, b.w.p0, r0);
  if (r1) copy_stream(m.w.p1, a.w.p1, b.w.p1, r1);
  if (r2) copy_stream(m.w.p2, a.w.p2, b.w.p2, r2);
  if (r3) copy_stream(m.w.p3, a.w.p3, b.w.p3, r3);
  HIP_CHECK(hipStreamSynchronize(stream_));
  return m;
}

void Engine::set_tensor(const std::string& name, int qt, int rows, int cols, const void* host, size_t nbytes) {
  const CuScope cu_scope(cus_);  // (grids sized to this engine's CU mask)
  if (finalized_) throw std::runtime_error("set_tensor after finalize");
  HIP_CHECK(hipSetDevice(cfg_.device));
  static const std::regex blk_re(R"(blk\.(\d+)\.(.+))");
  std::smatch m;
  if (name == "token_embd.weight") {
    tok_embd_ = upload_qmat(qt, rows, cols, host, nbytes);
    return;
  }
  if (name == "output.weight") {
    if (cfg_.vocab_parallel && rows != cfg_.vocab_size / cfg_.tp_size)
      throw std::runtime_error("vocab-parallel output.weight: expected " +
                               std::to_string(cfg_.vocab_size / cfg_.tp_size) + " rows (this rank's shard)");
    output_ = upload_qmat(qt, rows, cols, host, nbytes);
    return;
  }
  if (name == "output_norm.weight") {
    out_norm_ = upload_f32(host, (size_t)rows * cols, qt);
    return;
  }
  if (!std::regex_match(name, m, blk_re)) throw std::runtime_error("unknown tensor " + name);
  const int l = std::stoi(m[1]);
  if (l < 0 || l >= cfg_.n_layers) throw std::runtime_error("layer index out of range in " + name);
  const std::string t = m[2];
  LayerW& L = layers_[l];
  const size_t n = (size_t)rows * cols;
  if (t == "attn_norm.weight") L.attn_norm = upload_f32(host, n, qt);
  else if (t == "ffn_norm.weight") L.ffn_norm = upload_f32(host, n, qt);
  else if (t == "attn_q_norm.weight") L.q_norm = upload_f32(host, n, qt);
  else if (t == "attn_k_norm.weight") L.k_norm = upload_f32(host, n, qt);
  else if (t == "attn_q.weight") L.wq = upload_qmat(qt, rows, cols, host, nbytes);
  else if (t == "attn_k.weight") L.wk = upload_qmat(qt, rows, cols, host, nbytes);
  else if (t == "attn_v.weight") L.wv = upload_qmat(qt, rows, cols, host, nbytes);
  else if (t == "attn_output.weight") L.wo = upload_qmat(qt, rows, cols, host, nbytes);
  else if (t == "ffn_down.weight") L.wdown = upload_qmat(qt, rows, cols, host, nbytes);
  else if (t == "ffn_gate.weight" || t == "ffn_up.weight") {
    const std::string other = (t == "ffn_gate.weight") ? "ffn_up.weight" : "ffn_gate.weight";
    const std::string key = "blk." + std::to_string(l) + ".";
    QMat q = upload_qmat(qt, rows, cols, host, nbytes);
    auto it = pending_.find(key + other);
    if (it == pending_.end()) {
      pending_[key + t] = q;
    } else {
      const QMat& g = (t == "ffn_gate.weight") ? q : it->second;
      const QMat& u = (t == "ffn_gate.weight") ? it->second : q;
      L.wgu = interleave_rows(g, u);
      // the separate copies are no longer needed
      for (const QMat* mm : {&q, &it->second}) {
        auto pos = std::find(allocs_.begin(), allocs_.end(), mm->buf);
        if (pos != allocs_.end()) allocs_.erase(pos);
        weight_bytes_ -= mm->bytes;
        HIP_CHECK(hipFree(mm->buf));
      }
      pending_.erase(it);
    }
  } else if (t == "attn_q.bias" || t == "attn_k.bias" || t == "attn_v.bias") {
    const int qd = cfg_.n_heads * cfg_.head_dim, kvd = cfg_.n_kv_heads * cfg_.head_dim;
    if (!L.bqkv) {
      L.bqkv = (float*)dmalloc((size_t)(qd + 2 * kvd) * 4);
      HIP_CHECK(hipMemset(L.bqkv, 0, (size_t)(qd + 2 * kvd) * 4));
    }
    const int off = t == "attn_q.bias" ? 0 : (t == "attn_k.bias" ? qd : qd + kvd);
    float* tmp = upload_f32(host, n, qt);
    HIP_CHECK(hipMemcpy(L.bqkv + off, tmp, n * 4, hipMemcpyDeviceToDevice));
  } else {
    throw std::runtime_error("unknown layer tensor " + name);
  }
}

void Engine::init_random(const std::string& recipe_in, uint64_t seed) {
  const CuScope cu_scope(cus_);  // (grids sized to this engine's CU mask)
  TraceRange tr("aios.init_random");
  HIP_CHECK(hipSetDevice(cfg_.device));
  std::string r = recipe_in;
  std::transform(r.begin(), r.end(), r.begin(), ::toupper);
  const int d = cfg_.d_model, qd = cfg_.n_heads * cfg_.head_dim, kvd = cfg_.n_kv_heads * cfg_.head_dim;
  const int ff = cfg_.d_ff, V = cfg_.vocab_size, NL = cfg_.n_layers;
  auto more_bits = [&](int i) { return i < NL / 8 || i >= 7 * NL / 8 || (i - NL / 8) % 3 == 2; };
  auto type_for = [&](const std::string& t, int layer) -> int {
    if (r == "Q4_K_M") {
      if (t == "output") return QT_Q6_K;
      if (t == "attn_v" || t == "ffn_down") return more_bits(layer) ? QT_Q6_K : QT_Q4_K;
      return QT_Q4_K;
    }
    if (r == "Q5_K_M") {
      if (t == "output") return QT_Q6_K;
      if (t == "attn_v" || t == "ffn_down") return more_bits(layer) ? QT_Q6_K : QT_Q5_K;
      return QT_Q5_K;
    }
    if (r == "Q4_K") return QT_Q4_K;
    if (r == "Q6_K") return QT_Q6_K;
    if (r == "Q4_0") return t == "output" ? QT_Q6_K : QT_Q4_0;
    if (r == "Q8_0") return QT_Q8_0;
    if (r == "F16") return QT_F16;
    if (r == "BF16") return QT_BF16;
    // recipes whose formats the loader expands to bf16 (Q2_K / Q3_K / IQ4 / legacy 32-blocks): in HBM
    // their matrices ARE bf16, next to the native K-quants the mix keeps (models/config.py tensor_type)
    if (r == "Q3_K_M") {
      if (t == "output") return QT_Q6_K;
      if (t == "attn_v" || t == "ffn_down") return more_bits(layer) ? QT_Q5_K : QT_Q4_K;
      return t == "attn_output" ? QT_Q4_K : QT_BF16;
    }
    if (r == "Q2_K") {
      if (t == "output") return QT_Q6_K;
      return (t == "attn_v" || t == "ffn_down") && more_bits(layer) ? QT_Q4_K : QT_BF16;
    }
    if (r == "IQ4_NL" || r == "IQ4_XS" || r == "Q4_1" || r == "Q5_0" || r == "Q5_1") return t == "output" ? QT_Q6_K : QT_BF16;
    throw std::runtime_error("unknown recipe " + recipe_in);
  };
  uint64_t s = seed * 1000003ULL;
  auto mk = [&](int qt, int rows, int cols, float amp) {
    QMat m = alloc_qmat(qt, rows, cols);
    fill_random_weight(m.w, ++s, amp, stream_);
    return m;
  };
  auto vec = [&](int n, float base, float amp) {
    float* p = (float*)dmalloc((size_t)n * 4);
    weight_bytes_ += (size_t)n * 4;
    fill_random_f32(p, n, ++s, base, amp, stream_);
    return p;
  };
  const float amp = 0.02f;
  tok_embd_ = mk(type_for("token_embd", 0), V, d, 1.0f);
  if (!cfg_.tie_embeddings) output_ = mk(type_for("output", 0), cfg_.vocab_parallel ? V / cfg_.tp_size : V, d, amp);
  out_norm_ = vec(d, 1.f, 0.1f);
  for (int l = 0; l < NL; ++l) {
    LayerW& L = layers_[l];
    L.attn_norm = vec(d, 1.f, 0.1f);
    L.ffn_norm = vec(d, 1.f, 0.1f);
    if (cfg_.qk_norm) {
      L.q_norm = vec(cfg_.head_dim, 1.f, 0.1f);
      L.k_norm = vec(cfg_.head_dim, 1.f, 0.1f);
    }
    if (cfg_.qkv_bias) L.bqkv = vec(qd + 2 * kvd, 0.f, 0.02f);
    L.wq = mk(type_for("attn_q", l), qd, d, amp);
    L.wk = mk(type_for("attn_k", l), kvd, d, amp);
    L.wv = mk(type_for("attn_v", l), kvd, d, amp);
    L.wo = mk(type_for("attn_output", l), d, qd, amp);
    L.wgu = mk(type_for("ffn_gate", l), 2 * ff, d, amp);
    L.wdown = mk(type_for("ffn_down", l), d, ff, amp);
  }
  HIP_CHECK(hipStreamSynchronize(stream_));
}

std::vector<std::string> Engine::missing_tensors() const {
  std::vector<std::string> miss;
  if (!tok_embd_.valid()) miss.push_back("token_embd.weight");
  if (!out_norm_) miss.push_back("output_norm.weight");
  for (int l = 0; l < cfg_.n_layers; ++l) {
    const LayerW& L = layers_[l];
    const std::string p = "blk." + std::to_string(l) + ".";
    if (!L.attn_norm) miss.push_back(p + "attn_norm.weight");
    if (!L.ffn_norm) miss.push_back(p + "ffn_norm.weight");
    if (!L.wq.valid()) miss.push_back(p + "attn_q.weight");
    if (!L.wk.valid()) miss.push_back(p + "attn_k.weight");
    if (!L.wv.valid()) miss.push_back(p + "attn_v.weight");
    if (!L.wo.valid()) miss.push_back(p + "attn_output.weight");
    if (!L.wgu.valid()) miss.push_back(p + "ffn_gate.weight/ffn_up.weight");
    if (!L.wdown.valid()) miss.push_back(p + "ffn_down.weight");
    if (cfg_.qk_norm && (!L.q_norm || !L.k_norm)) miss.push_back(p + "attn_q_norm/attn_k_norm");
  }
  return miss;
}

std::string Engine::weight_type_summary() const {
  std::map<int, size_t> cnt;
  auto add = [&](const QMat& m) { if (m.valid()) cnt[m.w.qtype] += (size_t)m.w.rows * m.w.cols; };
  add(tok_embd_);
  add(output_);
  for (const LayerW& L : layers_) { add(L.wq); add(L.wk); add(L.wv); add(L.wo); add(L.wgu); add(L.wdown); }
  std::ostringstream os;
  for (auto& kv : cnt) os << kv.first << ":" << kv.second << " ";
  return os.str();
}

static std::vector<std::vector<const QMat*>> qkv_groups(const LayerW& L);

void Engine::finalize() {
  const CuScope cu_scope(cus_);  // (grids sized to this engine's CU mask)
  TraceRange tr("aios.finalize");
  HIP_CHECK(hipSetDevice(cfg_.device));
  stage_release();  // weights are in place: drop the load-time staging buffers
  auto miss = missing_tensors();
  if (!miss.empty()) throw std::runtime_error("missing tensors, first: " + miss[0]);
  if (!output_.valid()) {
    if (!cfg_.tie_embeddings) cfg_.tie_embeddings = 1;
    cfg_.vocab_parallel = 0;  // the tied table is the full vocabulary
    output_ = tok_embd_;  // tied embeddings (GGUF files without output.weight)
  }
  const int d = cfg_.d_model, hd = cfg_.head_dim, H = cfg_.n_heads, Hkv = cfg_.n_kv_heads;
  const int qd = H * hd, kvd = Hkv * hd, V = cfg_.vocab_size, Bm = cfg_.max_batch;
  if (cfg_.max_ctx % KV_BLOCK) cfg_.max_ctx = (int)align_up(cfg_.max_ctx, KV_BLOCK);  // whole KV blocks
  // paged KV pool: max_slots * max_ctx / KV_BLOCK blocks always suffice (a mapping or
  // un-sharing step never needs more distinct blocks than there are table entries) + one null
  // block that unmapped table entries point to on the device
  kv_maxb_ = cfg_.max_ctx / KV_BLOCK;
  kv_nblocks_ = cfg_.max_slots * kv_maxb_;
  bt_.assign((size_t)cfg_.max_slots * kv_maxb_, -1);
  refcnt_.assign(kv_nblocks_, 0);
  free_blocks_.clear();
  for (int b = kv_nblocks_ - 1; b >= 0; --b) free_blocks_.push_back(b);
  row_bt_host_.assign((size_t)Bm * kv_maxb_, kv_nblocks_);
  layer_kv_elems_ = (size_t)(kv_nblocks_ + 1) * Hkv * KV_BLOCK * hd;
  kv_es_ = cfg_.kv_fp8 ? 1 : 2;  // bytes per cached element (fp8 e4m3 or bf16)
  kv_bytes_ = 2 * layer_kv_elems_ * cfg_.n_layers * kv_es_;
  if (kv_scale_.size() != (size_t)2 * cfg_.n_layers) kv_scale_.assign((size_t)2 * cfg_.n_layers, 1.f);
  k_cache_ = (bf16_t*)dmalloc(kv_bytes_ / 2);
  v_cache_ = (bf16_t*)dmalloc(kv_bytes_ / 2);
  HIP_CHECK(hipMemset(k_cache_, 0, kv_bytes_ / 2));
  HIP_CHECK(hipMemset(v_cache_, 0, kv_bytes_ / 2));
  n_chunks_ = (cfg_.max_ctx + ATTN_CHUNK - 1) / ATTN_CHUNK;
  {
    const size_t nc = (size_t)std::max(prefill_rows_, Bm) * H;  // decode attention tickets [row][head]
    attn_cnt_ = (int*)dmalloc(nc * 4);
    HIP_CHECK(hipMemset(attn_cnt_, 0, nc * 4));
  }
  {
    const int half = hd / 2;
    std::vector<float> tab((size_t)cfg_.max_ctx * half * 2);
    for (int pos = 0; pos < cfg_.max_ctx; ++pos)
      for (int p = 0; p < half; ++p) {
        const double th = (double)pos * std::pow((double)cfg_.rope_theta, -2.0 * p / (double)hd);
        tab[((size_t)pos * half + p) * 2] = (float)std::cos(th);
        tab[((size_t)pos * half + p) * 2 + 1] = (float)std::sin(th);
      }
    rope_cs_ = (float2*)dmalloc(tab.size() * 4);
    HIP_CHECK(hipMemcpy(rope_cs_, tab.data(), tab.size() * 4, hipMemcpyHostToDevice));
  }

  size_t ws = 0;
  auto fbuf = [&](size_t n) { ws += n * 4; return (float*)dmalloc(n * 4); };
  auto ibuf = [&](size_t n) { ws += n * 4; int* p = (int*)dmalloc(n * 4); HIP_CHECK(hipMemset(p, 0, n * 4)); return p; };
  x_ = fbuf((size_t)Bm * d);
  q_ = fbuf((size_t)Bm * qd);
  qkv_ = fbuf((size_t)Bm * (qd + 2 * kvd));
  attn_ = fbuf((size_t)Bm * std::max(qd, d));
  ff_ = fbuf((size_t)Bm * std::max(cfg_.d_ff, d));
  // (the BF16 engine stages its x as bf16 whatever act_q8 says: the hand-off serves it too)
  if ((cfg_.act_q8 || layers_[0].wgu.w.qtype == QT_BF16) && cfg_.d_ff % 8 == 0 &&
      !(std::getenv("AIOS_FF16") && std::atoi(std::getenv("AIOS_FF16")) == 0)) {
    gv_ff16_ = (bf16_t*)dmalloc((size_t)Bm * cfg_.d_ff * 2);
    ws += (size_t)Bm * cfg_.d_ff * 2;
  }
  opart_ = fbuf((size_t)Bm * H * n_chunks_ * hd);
  ml_ = fbuf((size_t)Bm * H * n_chunks_ * 2);
  logits_ = fbuf((size_t)Bm * V);
  {
    // per-step decode parameters + grammar masks in ONE device block mirrored by a pinned host
    // block: a scheduler decode() uploads all of them with a single async copy (round 1 issued 8
    // pageable copies per step)
    const size_t mb = (size_t)Bm * ((V + 7) / 8);
    const size_t seeds_off = align_up(8 + (size_t)Bm * 4 * 7, 8);  // per-row seeds after the 7 row arrays
    par_mask_off_ = align_up(seeds_off + (size_t)Bm * 8, 256);
    par_bytes_ = par_mask_off_ + mb;
    d_par_ = (char*)dmalloc(par_bytes_);
    ws += par_bytes_;
    // two halves: the pipelined decode writes step t+1's parameters while step t's copy may still be
    // queued (decode_submit); the other paths use the first half
    HIP_CHECK(hipHostMalloc(&h_par_, 2 * par_bytes_, hipHostMallocDefault));
    HIP_CHECK(hipHostMalloc((void**)&h_mask_, mb, hipHostMallocDefault));
    HIP_CHECK(hipEventCreateWithFlags(&pipe_ev_, hipEventDisableTiming));
    HIP_CHECK(hipHostMalloc((void**)&h_tok_out_, (size_t)Bm * 4, hipHostMallocDefault));
    std::memset(h_par_, 0, 2 * par_bytes_);
    d_seed_ = (uint64_t*)d_par_;
    d_slot_ = (int*)(d_par_ + 8);
    d_tokens_ = d_slot_ + Bm;
    d_pos_ = d_tokens_ + Bm;
    d_seqlen_ = d_pos_ + Bm;
    d_topk_ = d_seqlen_ + Bm;
    d_temp_ = (float*)(d_topk_ + Bm);
    d_topp_ = d_temp_ + Bm;
    d_seeds_ = (uint64_t*)(d_par_ + seeds_off);
    d_mask_ = (uint8_t*)(d_par_ + par_mask_off_);
    float* htp = (float*)(h_par_ + 8) + 6 * (size_t)Bm;
    for (int b = 0; b < Bm; ++b) htp[b] = 1.f;
    HIP_CHECK(hipMemcpy(d_par_, h_par_, par_bytes_, hipMemcpyHostToDevice));
  }
  d_bt_ = ibuf((size_t)cfg_.max_slots * kv_maxb_);
  d_row_bt_ = ibuf((size_t)Bm * kv_maxb_);
  {
    std::vector<int> nul((size_t)cfg_.max_slots * kv_maxb_, kv_nblocks_);
    HIP_CHECK(hipMemcpy(d_bt_, nul.data(), nul.size() * 4, hipMemcpyHostToDevice));
    HIP_CHECK(hipMemcpy(d_row_bt_, nul.data(), (size_t)Bm * kv_maxb_ * 4, hipMemcpyHostToDevice));
  }
  attn_bt_ = d_row_bt_;
  attn_bt_rows_ = 1;
  d_step_ = ibuf(4);
  d_step_kv_ = ibuf((size_t)Bm * 2);
  d_step_rope_ = (float2*)fbuf((size_t)Bm * hd);
  d_fpos_ = ibuf(4);
  sample_ws_bytes_ = sample_ws_bytes(Bm, V);
  sample_ws_ = dmalloc(sample_ws_bytes_);
  ws += sample_ws_bytes_;
  sample_cnt_ = ibuf(Bm);
  d_history_ = ibuf((size_t)Bm * (cfg_.max_ctx + 1));
  const int R = prefill_rows_;
  pf_x_ = fbuf((size_t)R * d);
  pf_q_ = fbuf((size_t)R * qd);
  pf_qkv_ = fbuf((size_t)R * (qd + 2 * kvd));
  pf_attn_ = fbuf((size_t)R * std::max(qd, d));
  pf_ff_ = fbuf((size_t)R * std::max(cfg_.d_ff, d));
  pf_opart_ = fbuf((size_t)R * H * n_chunks_ * hd);
  pf_ml_ = fbuf((size_t)R * H * n_chunks_ * 2);
  pf_a16_ = (bf16_t*)dmalloc((size_t)R * std::max({d, qd, cfg_.d_ff}) * 2);
  pf_tokens_ = ibuf(R);
  pf_pos_ = ibuf(R);
  pf_seqlen_ = ibuf(R);
  pf_slot_ = ibuf(R);
  // GEMM prefill path: supported when every projection is a GEMM format with 64-aligned shapes
  // and the head layout has a flash-attention instantiation
  {
    if (const char* e = std::getenv("AIOS_PREFILL_GEMM_MIN")) gm_min_rows_ = std::max(1, std::atoi(e));
    // one chunk per prompt up to 2048 tokens: the M tile count, not the chunk count, fills the chip
    gm_rows_ = std::min(cfg_.max_ctx, 2048);
    if (const char* e = std::getenv("AIOS_PREFILL_GEMM_ROWS")) gm_rows_ = std::max(64, std::atoi(e));
    bool ok = attn_prefill_supports(H, Hkv, hd) && d % 64 == 0 && cfg_.d_ff % 64 == 0 && qd % 64 == 0 && kvd % 64 == 0;
    for (const auto& L : layers_) {
      for (const QMat* m : {&L.wq, &L.wk, &L.wv, &L.wo, &L.wgu, &L.wdown})
        if (!gemm_supports(m->w.qtype) || m->w.rows % 64 || m->w.cols % 64) ok = false;
    }
    if (const char* e = std::getenv("AIOS_PREFILL_GEMM"))
      if (std::atoi(e) == 0) ok = false;
    gm_ok_ = ok;
    if (ok) {
      const int G = gm_rows_;
      gm_x_ = fbuf((size_t)G * d);
      gm_qkv_ = fbuf((size_t)G * (qd + 2 * kvd));
      gm_q_ = fbuf((size_t)G * qd);
      gm_part_ = fbuf((size_t)G * d);
      gm_a16_ = (bf16_t*)dmalloc((size_t)G * d * 2);
      gm_ff16_ = (bf16_t*)dmalloc((size_t)G * cfg_.d_ff * 2);
      gm_attn16_ = (bf16_t*)dmalloc((size_t)G * qd * 2);
      ws += (size_t)G * (d + cfg_.d_ff + qd) * 2;
      gm_tokens_ = ibuf(G);
      gm_pos_ = ibuf(G);
      gm_slot_ = ibuf(G);
      if (const char* e = std::getenv("AIOS_DECODE_GEMM_MIN_B")) {
        dec_gemm_min_b_ = std::atoi(e);
      } else {
        // B rows go through the B-row LDS-DMA engine only if EVERY projection's LDS plan fits at that
        // B; where one does not (e.g. a 28672-wide down projection at B = 4: 115 KB of staged x), the
        // row-pair fallback is 2-3x slower than the skinny GEMM, so that B takes the GEMM path
        // (ADVICE r3).  Also bounds the short-prompt prefill rows that use the GEMV path.
        for (int b = 2; b < dec_gemm_min_b_ && b <= Bm; ++b) {
          bool ok = true;
          for (int l = 0; l < cfg_.n_layers && ok; ++l) {
            const LayerW& L = layers_[l];
            for (auto& grp : qkv_groups(L)) {
              int n = 0;
              for (auto* m : grp) n += m->w.rows;
              ok = ok && gemv_engine_fits(gemv_args(grp, n, d, b, x_, d, L.attn_norm, q_, n, EPI_STORE, l));
            }
            ok = ok && gemv_engine_fits(gemv_args({&L.wo}, d, qd, b, attn_, qd, nullptr, x_, d, EPI_RESID, l)) &&
                 gemv_engine_fits(gemv_args({&L.wgu}, 2 * cfg_.d_ff, d, b, x_, d, L.ffn_norm, ff_, cfg_.d_ff,
                                            EPI_SWIGLU, l)) &&
                 gemv_engine_fits(gemv_args({&L.wdown}, d, cfg_.d_ff, b, ff_, cfg_.d_ff, nullptr, x_, d, EPI_RESID, l));
          }
          if (!ok) {
            dec_gemm_min_b_ = b;
            gm_min_rows_ = std::min(gm_min_rows_, b);
          }
        }
      }
      // split-K slabs + tickets for every skinny-GEMM call: batched decode (M <= max_batch, the
      // lm_head included) AND prefill chunks of 16-64 tokens (no lm_head) -- sized for the batch
      // only, a 32-token prompt ran its projections unsplit (32 workgroups for N = d_model)
      const int maxN = std::max({qd + 2 * kvd, d, 2 * cfg_.d_ff, V});
      const int maxN_pf = std::max({qd + 2 * kvd, d, 2 * cfg_.d_ff});
      gk_ws_bytes_ = std::max(Bm >= 2 ? gemm_skinny_ws_bytes(std::min(Bm, 64), maxN) : (size_t)0,
                              gemm_skinny_ws_bytes(64, maxN_pf));
      gk_ws_ = (float*)dmalloc(gk_ws_bytes_);
      ws += gk_ws_bytes_;
      gk_cnt_len_ = gemm_skinny_cnt_len(maxN);
      gk_cnt_ = ibuf(gk_cnt_len_);
      if (const char* e = std::getenv("AIOS_GEMM_NORM_FUSE")) nrm_fuse_ = std::atoi(e);
      {  // split-RMSNorm operands of short (<= 64-row) prefill chunks, independent of max_batch
        GemmQArgs p;
        std::memset(&p, 0, sizeof(p));
        p.M = 64; p.N = d; p.K = d; p.nseg = 1; p.seg[0] = layers_[0].wo.w;
        const int parts = gemm_skinny_ntile(p);
        if (nrm_fuse_ && parts > 0 && parts % 4 == 0 && parts <= 64 && d % 128 == 0) {
          const int Gs = std::min(G, 64);
          gm_nparts_ = parts;
          gm_xn16_ = (bf16_t*)dmalloc((size_t)Gs * d * 2);
          gm_npart_ = fbuf((size_t)Gs * parts);
          ws += (size_t)Gs * d * 2;
        }
      }
      if (Bm >= 2) {
        dec_a16_ = (bf16_t*)dmalloc((size_t)Bm * std::max(d, qd) * 2);
        dec_ff16_ = (bf16_t*)dmalloc((size_t)Bm * cfg_.d_ff * 2);
        ws += (size_t)Bm * (std::max(d, qd) + cfg_.d_ff) * 2;
        GemmQArgs p;  // the residual producer's shape (O / down: N = d_model, one segment)
        std::memset(&p, 0, sizeof(p));
        p.M = std::min(Bm, 64); p.N = d; p.K = d; p.nseg = 1; p.seg[0] = layers_[0].wo.w;
        const int parts = gemm_skinny_ntile(p);
        if (nrm_fuse_ && Bm <= 64 && parts > 0 && parts % 4 == 0 && parts <= 64 && d % 128 == 0) {
          nrm_parts_ = parts;
          dec_xn16_ = (bf16_t*)dmalloc((size_t)Bm * d * 2);
          nrm_part_ = fbuf((size_t)Bm * parts);
          ws += (size_t)Bm * d * 2;
        }
        // TP: the all-reduce after O / down writes the next GEMM's split-norm operand itself
        if (cfg_.tp_size > 1 && dec_xn16_ && resid_norm_parts(d) > 0 && resid_norm_parts(d) <= 64) {
          tpn_parts_ = resid_norm_parts(d);
          tpn_part_ = fbuf((size_t)Bm * tpn_parts_);
        }
      }
    }
  }
  ws_bytes_ = ws;
  HIP_CHECK(hipDeviceSynchronize());
  tune_prefill_gemm();
  finalized_ = true;
}

// Measured prefill-GEMM plans (kernels/gemm_pf.hip): every distinct projection launch of this model
// -- QKV stack, O, gate/up (SwiGLU), down, per weight-format signature -- timed over its candidate
// tiles / K splits at M = 64 .. gm_rows_ (powers of two), the fastest kept per M bucket in the
// process-wide plan cache (one tuning per shape per process; ~0.3 s for Mistral-7B).  Activations
// are random bf16 (a zero fill clocks the chip differently).  AIOS_GEMM_PF_TUNE=0: model plans only.
void Engine::tune_prefill_gemm() {
  if (!gm_ok_ || cfg_.n_layers == 0) return;
  if (const char* e = std::getenv("AIOS_GEMM_PF_TUNE"))
    if (std::atoi(e) == 0) return;
  const int d = cfg_.d_model, hd = cfg_.head_dim, qd = cfg_.n_heads * hd, kvd = cfg_.n_kv_heads * hd;
  const int ff = cfg_.d_ff, G = gm_rows_, ldqkv = qd + 2 * kvd;
  const bool tp = cfg_.tp_size > 1;
  const size_t n = (size_t)G * std::max({d, qd, ff});
  float* tmp = nullptr;
  HIP_CHECK(hipMalloc(&tmp, n * 4));
  fill_random_f32(tmp, n, 0x7u, 0.f, 1.f, stream_);
  launch_f32_to_bf16(tmp, gm_a16_, (size_t)G * d, stream_);
  launch_f32_to_bf16(tmp, gm_attn16_, (size_t)G * qd, stream_);
  launch_f32_to_bf16(tmp, gm_ff16_, (size_t)G * ff, stream_);
  std::set<std::string> seen;
  for (int M = 64; M <= G; M *= 2) {
    for (const LayerW& L : layers_) {
      auto tune = [&](GemmQArgs& g, const char* what) {
        std::string sig = std::string(what) + ":" + std::to_string(M);
        for (int s = 0; s < g.nseg; ++s) sig += "," + std::to_string(g.seg[s].qtype);
        if (!seen.insert(sig).second) return;
        gemm_pf_autotune(g, stream_);
      };
      GemmQArgs g;
      std::memset(&g, 0, sizeof(g));
      g.A = gm_a16_; g.lda = d; g.M = M; g.K = d; g.nseg = 3;
      g.seg[0] = L.wq.w; g.seg[1] = L.wk.w; g.seg[2] = L.wv.w;
      g.seg_n0[0] = 0; g.seg_n0[1] = qd; g.seg_n0[2] = qd + kvd;
      g.N = ldqkv; g.C = gm_qkv_; g.ldc = ldqkv; g.epi = GEPI_STORE;
      tune(g, "qkv");
      std::memset(&g, 0, sizeof(g));
      g.A = gm_attn16_; g.lda = qd; g.M = M; g.K = qd; g.nseg = 1; g.seg[0] = L.wo.w; g.N = d; g.ldc = d;
      if (tp) { g.C = gm_part_; g.epi = GEPI_STORE; } else { g.C = gm_x_; g.epi = GEPI_ACCUM; }
      tune(g, "o");
      std::memset(&g, 0, sizeof(g));
      g.A = gm_a16_; g.lda = d; g.M = M; g.K = d; g.nseg = 1; g.seg[0] = L.wgu.w; g.N = 2 * ff;
      g.C16 = gm_ff16_; g.ldc = ff; g.epi = GEPI_SWIGLU_BF16;
      tune(g, "gu");
      std::memset(&g, 0, sizeof(g));
      g.A = gm_ff16_; g.lda = ff; g.M = M; g.K = ff; g.nseg = 1; g.seg[0] = L.wdown.w; g.N = d; g.ldc = d;
      if (tp) { g.C = gm_part_; g.epi = GEPI_STORE; } else { g.C = gm_x_; g.epi = GEPI_ACCUM; }
      tune(g, "down");
    }
  }
  HIP_CHECK(hipStreamSynchronize(stream_));
  HIP_CHECK(hipFree(tmp));
}

// TP: sum the row-parallel partials in `p` over the ranks and add the total into `residual`
// (one fused launch: xGMI one-shot all-reduce + residual add, aios_amd/csrc/comm.h)
void Engine::allreduce(float* p, size_t n, float* residual) {
  if (cfg_.tp_size > 1) {
    if (!allreduce_) throw std::runtime_error("tensor-parallel engine without an all-reduce hook");
    allreduce_(allreduce_ctx_, p, n, residual, stream_);
  }
}

// decode GEMV tuning knobs from the environment (read once): AIOS_GEMV_{U,GRID,KSPLIT}_{QKV,O,GU,DOWN,LM}
// -- in-situ sweeps of the captured decode step (tools/gemv_knob_sweep.sh); 0 = the launcher's choice
static int gemv_knob(const char* what, const char* kind) {
  static std::map<std::string, int> cache;
  const std::string key = std::string("AIOS_GEMV_") + what + "_" + kind;
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  const char* e = std::getenv(key.c_str());
  const int v = e ? std::atoi(e) : 0;
  cache[key] = v;
  return v;
}
static void apply_knobs(GemvArgs& a, const char* kind) {
  a.tune_u = gemv_knob("U", kind);
  a.tune_grid = gemv_knob("GRID", kind);
  a.tune_ksplit = gemv_knob("KSPLIT", kind);
}

void Engine::gemv(const std::vector<const QMat*>& segs, int N, int K, int B, const float* x, int ldx,
                  const float* norm_w, float* y, int ldy, int epi, int layer) {
  launch_gemv(gemv_args(segs, N, K, B, x, ldx, norm_w, y, ldy, epi, layer), stream_);
}

GemvArgs Engine::gemv_args(const std::vector<const QMat*>& segs, int N, int K, int B, const float* x, int ldx,
                           const float* norm_w, float* y, int ldy, int epi, int layer) {
  GemvArgs a;
  std::memset(&a, 0, sizeof(a));
  a.act_q8 = cfg_.act_q8;
  a.nseg = (int)segs.size();
  int row = 0;
  for (int s = 0; s < a.nseg; ++s) {
    a.seg[s] = segs[s]->w;
    a.seg_row0[s] = row;
    row += segs[s]->w.rows;
  }
  a.N = N;
  a.K = K;
  a.B = B;
  a.row_base = 0;
  a.x = x;
  a.ldx = ldx;
  a.norm_w = norm_w;
  a.eps = cfg_.norm_eps;
  a.y = y;
  a.ldy = ldy;
  a.epi = epi;
  if (epi == EPI_QKV) {
    const LayerW& L = layers_[layer];
    a.bias = L.bqkv;
    a.head_dim = cfg_.head_dim;
    a.q_dim = cfg_.n_heads * cfg_.head_dim;
    a.kv_dim = cfg_.n_kv_heads * cfg_.head_dim;
    a.n_kv_heads = cfg_.n_kv_heads;
    a.max_ctx = cfg_.max_ctx;
    a.rope_neox = cfg_.rope_neox;
    a.rope_base = cfg_.rope_theta;
    a.rope_cs = rope_cs_;
    a.k_cache = kv_layer(k_cache_, layer);
    a.v_cache = kv_layer(v_cache_, layer);
    kv_write_args(a, layer);
  }
  apply_knobs(a, K == cfg_.d_ff ? "DOWN" : (N == 2 * cfg_.d_ff ? "GU" : (N == cfg_.vocab_size ? "LM" : "O")));
  return a;
}

// QKV segments: group into launches where only the last segment may differ in format
static std::vector<std::vector<const QMat*>> qkv_groups(const LayerW& L) {
  const QMat* s[3] = {&L.wq, &L.wk, &L.wv};
  if (s[0]->w.qtype == s[1]->w.qtype && gemv_supports(s[0]->w.qtype, s[2]->w.qtype)) return {{s[0], s[1], s[2]}};
  if (s[0]->w.qtype == s[1]->w.qtype) return {{s[0], s[1]}, {s[2]}};
  return {{s[0]}, {s[1]}, {s[2]}};
}

void Engine::gemm(GemmQArgs& g) {
  g.ws = gk_ws_;
  g.ws_bytes = gk_ws_bytes_;
  g.cnt = gk_cnt_;
  g.cnt_len = gk_cnt_len_;
  launch_gemm_q(g, stream_);
}

// one transformer block for the B rows staged in x_ (decode) -- also used by prefill with
// pointers swapped in (see prefill()).
// Batched decode (B >= dec_gemm_min_b_): the int8 GEMV's dot work grows with B while the weight
// stream does not, so from two concurrent sequences on the projections go through the skinny
// MFMA GEMM (weights dequantised once per step into MFMA operands, split-K reduced in-launch),
// with explicit RMSNorm -> bf16 and RoPE/KV-write launches in place of the GEMV prologue /
// epilogue fusions.  SwiGLU runs in the gate/up GEMM's epilogue (bf16 out for the down GEMM).
bool Engine::nrm_on(int B) const { return nrm_parts_ > 0 && dec_xn16_ && cfg_.tp_size == 1 && B <= 64; }
// AIOS_TP_NORM_FUSE=0 restores the separate RMSNorm launches after C1 / C2 (A/B and tests)
bool Engine::tpn_on(int B) const {
  static const bool on = !(std::getenv("AIOS_TP_NORM_FUSE") && std::atoi(std::getenv("AIOS_TP_NORM_FUSE")) == 0);
  return on && tpn_parts_ > 0 && allreduce_norm_ && cfg_.tp_size > 1 && B <= 64;
}

void Engine::layer_decode_gemm(int l, int B) {
  const LayerW& L = layers_[l];
  const int d = cfg_.d_model, hd = cfg_.head_dim, H = cfg_.n_heads, Hkv = cfg_.n_kv_heads, ff = cfg_.d_ff;
  const int qd = H * hd, kvd = Hkv * hd, ldqkv = qd + 2 * kvd;
  const bool tp = cfg_.tp_size > 1;
  const bool fn = nrm_on(B);
  const bool tpn = tp && tpn_on(B);  // (fn and tpn are exclusive: fn needs tp_size 1)
  bf16_t* kc = kv_layer(k_cache_, l);
  bf16_t* vc = kv_layer(v_cache_, l);
  // consumer side of the split RMSNorm: A = bf16(x * g) from the previous residual GEMM
  auto nrm_in = [&](GemmQArgs& g) {
    g.A = dec_xn16_; g.nrm_in = nrm_part_; g.nrm_parts = nrm_parts_; g.nrm_eps = cfg_.norm_eps;
  };
  // producer side: residual add + bf16(x_new * g_next) + per-tile sums of squares
  auto nrm_out = [&](GemmQArgs& g, const float* g_next) {
    g.epi = GEPI_ACCUM_NORM; g.nrm_g = g_next; g.nrm_out16 = dec_xn16_; g.nrm_part = nrm_part_;
    g.nrm_parts = nrm_parts_;
  };
  // TP: the same contract, produced by the fused all-reduce (C1 / C2) into tpn_part_
  auto tpn_in = [&](GemmQArgs& g) {
    g.A = dec_xn16_; g.nrm_in = tpn_part_; g.nrm_parts = tpn_parts_; g.nrm_eps = cfg_.norm_eps;
  };
  auto tp_reduce = [&](float* part, const float* g_next) {
    if (tpn) allreduce_norm_(allreduce_norm_ctx_, part, B, d, x_, ResidNorm{g_next, dec_xn16_, d, tpn_part_, tpn_parts_},
                             stream_);
    else allreduce(part, (size_t)B * d, x_);
  };
  if (!((fn || tpn) && l > 0)) launch_rmsnorm_bf16(x_, d, L.attn_norm, dec_a16_, d, B, d, cfg_.norm_eps, stream_);
  GemmQArgs g;
  std::memset(&g, 0, sizeof(g));
  g.A = dec_a16_; g.lda = d; g.M = B; g.K = d; g.nseg = 3;
  if (fn && l > 0) nrm_in(g);
  if (tpn && l > 0) tpn_in(g);
  g.seg[0] = L.wq.w; g.seg[1] = L.wk.w; g.seg[2] = L.wv.w;
  g.seg_n0[0] = 0; g.seg_n0[1] = qd; g.seg_n0[2] = qd + kvd;
  g.N = ldqkv; g.C = qkv_; g.ldc = ldqkv; g.epi = GEPI_STORE;
  // RoPE + q store + KV-cache write in the GEMM epilogue (one launch per layer less) whenever
  // qkv_post would only do that (non-NeoX pairs, no QK-norm, no QKV bias)
  static const int qkv_epi_max_b = [] {
    const char* e = std::getenv("AIOS_GEMM_QKV_EPI_MAX_B");
    return e ? std::atoi(e) : 64;
  }();
  const bool qkv_epi = !cfg_.qk_norm && !cfg_.rope_neox && !L.bqkv && rope_cs_ && B <= qkv_epi_max_b;
  if (qkv_epi) {
    g.epi = GEPI_QKV; g.col0 = 0;
    g.head_dim = hd; g.q_dim = qd; g.kv_dim = kvd; g.n_kv_heads = Hkv; g.max_ctx = cfg_.max_ctx;
    g.rope_cs = rope_cs_; g.pos = d_pos_; g.slot = d_slot_; g.block_table = d_bt_;
    g.q_out = q_; g.k_cache = kc; g.v_cache = vc;
    kv_write_args(g, l);
  }
  gemm(g);
  static const bool attn_out16 = !(std::getenv("AIOS_ATTN_OUT16") && std::atoi(std::getenv("AIOS_ATTN_OUT16")) == 0);
  if (!qkv_epi) {
  QkvPostArgs p;
  p.qkv = qkv_; p.ldqkv = ldqkv; p.T = B;
  p.n_heads = H; p.n_kv_heads = Hkv; p.head_dim = hd;
  p.bias = L.bqkv; p.q_norm = L.q_norm; p.k_norm = L.k_norm; p.eps = cfg_.norm_eps;
  p.rope_neox = cfg_.rope_neox; p.rope_base = cfg_.rope_theta; p.rope_cs = rope_cs_;
  p.pos = d_pos_; p.slot = d_slot_; p.q_out = q_;
  p.k_cache = kc; p.v_cache = vc; p.max_ctx = cfg_.max_ctx; p.block_table = d_bt_;
  kv_write_args(p, l);
  launch_qkv_post(p, stream_);
  }
  {
    AttnDecodeArgs a;
    a.split = 0;
    a.q = q_; a.k_cache = kc; a.v_cache = vc; a.seq_len = d_seqlen_; a.slot = d_slot_;
    kv_read_args(a, l);
    a.block_table = attn_bt_; a.bt_rows = attn_bt_rows_;
    a.B = B; a.n_heads = H; a.n_kv_heads = Hkv; a.head_dim = hd; a.max_ctx = cfg_.max_ctx;
    a.n_chunks = n_chunks_; a.scale = 1.f / std::sqrt((float)hd);
    a.o_part = opart_; a.ml = ml_; a.out = attn_; a.counters = attn_cnt_;
    if (attn_out16) a.out16 = dec_a16_;  // bf16 straight from the attention epilogue (no conversion launch)
    launch_attn_decode(a, stream_);
  }
  if (!attn_out16) launch_f32_to_bf16(attn_, dec_a16_, (size_t)B * qd, stream_);
  std::memset(&g, 0, sizeof(g));
  g.A = dec_a16_; g.lda = qd; g.M = B; g.K = qd; g.nseg = 1; g.seg[0] = L.wo.w; g.N = d; g.ldc = d;
  if (tp) { g.C = ff_; g.epi = GEPI_STORE; } else { g.C = x_; g.epi = GEPI_ACCUM; }
  if (fn) nrm_out(g, L.ffn_norm);
  gemm(g);
  if (tp) tp_reduce(ff_, L.ffn_norm);
  if (!fn && !tpn) launch_rmsnorm_bf16(x_, d, L.ffn_norm, dec_a16_, d, B, d, cfg_.norm_eps, stream_);
  std::memset(&g, 0, sizeof(g));
  g.A = dec_a16_; g.lda = d; g.M = B; g.K = d; g.nseg = 1; g.seg[0] = L.wgu.w; g.N = 2 * ff;
  g.C16 = dec_ff16_; g.ldc = ff; g.epi = GEPI_SWIGLU_BF16;
  if (fn) nrm_in(g);
  if (tpn) tpn_in(g);
  gemm(g);
  std::memset(&g, 0, sizeof(g));
  g.A = dec_ff16_; g.lda = ff; g.M = B; g.K = ff; g.nseg = 1; g.seg[0] = L.wdown.w; g.N = d; g.ldc = d;
  if (tp) { g.C = attn_; g.epi = GEPI_STORE; } else { g.C = x_; g.epi = GEPI_ACCUM; }
  // the next consumer: layer l + 1's QKV, or the lm_head after the last layer
  const float* g_next = l + 1 < cfg_.n_layers ? layers_[l + 1].attn_norm : out_norm_;
  if (fn) nrm_out(g, g_next);
  nrm_lm_ = (fn || tpn) && l + 1 == cfg_.n_layers;
  lm_nrm_in_ = tpn ? tpn_part_ : nrm_part_;
  lm_nrm_parts_ = tpn ? tpn_parts_ : nrm_parts_;
  gemm(g);
  if (tp) tp_reduce(attn_, g_next);
}

void Engine::layer_decode(int l, int B) {
  if (dec_a16_ && ((dec_gemm_min_b_ > 0 && B >= dec_gemm_min_b_) || B > 8)) {
    layer_decode_gemm(l, B);
    return;
  }
  if (B > 8) throw std::runtime_error("decode: batches above 8 need the GEMM path (GEMM-capable weights)");
  const LayerW& L = layers_[l];
  const int d = cfg_.d_model, hd = cfg_.head_dim, qd = cfg_.n_heads * hd, kvd = cfg_.n_kv_heads * hd;
  const bool fused_qkv = !cfg_.qk_norm && !cfg_.rope_neox;
  auto qkv_args = [&](const std::vector<const QMat*>& grp, int row0) {
    int n = 0;
    for (auto* m : grp) n += m->w.rows;
    GemvArgs a;
    std::memset(&a, 0, sizeof(a));
    a.act_q8 = cfg_.act_q8;
    a.nseg = (int)grp.size();
    int r = 0;
    for (int s = 0; s < a.nseg; ++s) { a.seg[s] = grp[s]->w; a.seg_row0[s] = r; r += grp[s]->w.rows; }
    a.N = n; a.K = d; a.B = B; a.row_base = row0;
    a.x = x_; a.ldx = d; a.norm_w = L.attn_norm; a.eps = cfg_.norm_eps;
    if (fused_qkv) {
      a.epi = EPI_QKV; a.y = q_; a.ldy = qd;
      a.bias = L.bqkv;
      a.head_dim = hd; a.q_dim = qd; a.kv_dim = kvd; a.n_kv_heads = cfg_.n_kv_heads; a.max_ctx = cfg_.max_ctx;
      a.rope_neox = cfg_.rope_neox; a.rope_base = cfg_.rope_theta; a.rope_cs = rope_cs_;
      a.pos = d_pos_; a.slot = d_slot_;
      a.k_cache = kv_layer(k_cache_, l);
      a.v_cache = kv_layer(v_cache_, l);
      kv_write_args(a, l);
      a.block_table = d_bt_;
      if (step_prep_on_ && B == 1) { a.step_kv = d_step_kv_; a.step_rope = d_step_rope_; }
    } else {
      a.epi = EPI_STORE; a.y = qkv_; a.ldy = qd + 2 * kvd;
    }
    apply_knobs(a, "QKV");
    static const int qkv_dbg = [] {  // probes only (AIOS_QKV_DBG=0x20000: epilogue lookups skipped)
      const char* e = std::getenv("AIOS_QKV_DBG");
      return e ? (int)std::strtol(e, nullptr, 0) : 0;
    }();
    a.tune_dbg = qkv_dbg;
    return a;
  };
  // ---- QKV (+RMSNorm prologue, RoPE + KV-cache epilogue)
  {
    int row0 = 0;
    for (auto& grp : qkv_groups(L)) {
      const GemvArgs a = qkv_args(grp, row0);
      launch_gemv(a, stream_);
      row0 += a.N;
    }
    if (!fused_qkv) {
      if (L.bqkv) throw std::runtime_error("qkv bias with unfused QKV path not supported yet");
      QkvPostArgs p;
      p.qkv = qkv_; p.ldqkv = qd + 2 * kvd; p.T = B;
      p.n_heads = cfg_.n_heads; p.n_kv_heads = cfg_.n_kv_heads; p.head_dim = hd;
      p.q_norm = L.q_norm; p.k_norm = L.k_norm; p.eps = cfg_.norm_eps;
      p.rope_neox = cfg_.rope_neox; p.rope_base = cfg_.rope_theta; p.rope_cs = rope_cs_;
      p.pos = d_pos_; p.slot = d_slot_; p.q_out = q_;
      p.k_cache = kv_layer(k_cache_, l);
      p.v_cache = kv_layer(v_cache_, l);
      kv_write_args(p, l);
      p.max_ctx = cfg_.max_ctx;
      p.block_table = d_bt_;
      launch_qkv_post(p, stream_);
    }
  }
  // ---- attention (fp32 output: a bf16 hand-off to O measured neutral, 544.0-544.5 vs 545.0-545.7 tok/s)
  {
    AttnDecodeArgs a;
    a.split = 0;
    a.q = q_;
    a.k_cache = kv_layer(k_cache_, l);
    a.v_cache = kv_layer(v_cache_, l);
    kv_read_args(a, l);
    a.seq_len = d_seqlen_;
    a.slot = d_slot_;
    a.block_table = attn_bt_; a.bt_rows = attn_bt_rows_;
    a.B = B; a.n_heads = cfg_.n_heads; a.n_kv_heads = cfg_.n_kv_heads; a.head_dim = hd; a.max_ctx = cfg_.max_ctx;
    a.n_chunks = n_chunks_;
    a.scale = 1.f / std::sqrt((float)hd);
    a.o_part = opart_; a.ml = ml_; a.out = attn_; a.counters = attn_cnt_;
    launch_attn_decode(a, stream_);
  }
  // ---- O projection (+ residual; TP: partial -> all-reduce -> add, fused into the GEMV epilogue
  // when the comm provides it)
  {
    const bool tp = cfg_.tp_size > 1;
    if (!(tp && tp_fuse_gemv(gemv_args({&L.wo}, d, qd, B, attn_, qd, nullptr, x_, d, EPI_TP_RESID, l)))) {
      GemvArgs a = gemv_args({&L.wo}, d, qd, B, attn_, qd, nullptr, tp ? ff_ : x_, d, tp ? EPI_STORE : EPI_RESID, l);
      launch_gemv(a, stream_);
      if (tp) allreduce(ff_, (size_t)B * d, x_);
    }
  }
  // ---- gate/up (+RMSNorm, SwiGLU; bf16 out when the down GEMV stages int8 activations, i.e. both
  // matrices take the int8-activation kernels: quantised formats, not F16 / BF16)
  auto q8k = [](int qt) { return qt != QT_F16 && qt != QT_BF16 && qt != QT_F32; };
  bf16_t* ff16 = (gv_ff16_ && q8k(L.wgu.w.qtype) && q8k(L.wdown.w.qtype)) ? gv_ff16_ : nullptr;
  if (gv_ff16_ && L.wgu.w.qtype == QT_BF16 && L.wdown.w.qtype == QT_BF16 &&
      gemv_bf16_engine_fits(gemv_args({&L.wgu}, 2 * cfg_.d_ff, d, B, x_, d, L.ffn_norm, ff_, cfg_.d_ff, EPI_SWIGLU, l)) &&
      gemv_bf16_engine_fits(gemv_args({&L.wdown}, d, cfg_.d_ff, B, ff_, cfg_.d_ff, nullptr, x_, d, EPI_RESID, l)))
    ff16 = gv_ff16_;  // BF16 weights: both GEMVs on the BF16 engine, which reads / writes the bf16 hand-off
  {
    GemvArgs a = gemv_args({&L.wgu}, 2 * cfg_.d_ff, d, B, x_, d, L.ffn_norm, ff_, cfg_.d_ff, EPI_SWIGLU, l);
    a.y16 = ff16;
    launch_gemv(a, stream_);
  }
  // ---- down (+ residual)
  {
    const bool tp = cfg_.tp_size > 1;
    GemvArgs f = gemv_args({&L.wdown}, d, cfg_.d_ff, B, ff_, cfg_.d_ff, nullptr, x_, d, EPI_TP_RESID, l);
    f.x16 = ff16;
    if (!(tp && tp_fuse_gemv(f))) {
      GemvArgs a = gemv_args({&L.wdown}, d, cfg_.d_ff, B, ff_, cfg_.d_ff, nullptr, tp ? attn_ : x_, d,
                             tp ? EPI_STORE : EPI_RESID, l);
      a.x16 = ff16;
      launch_gemv(a, stream_);
      if (tp) allreduce(attn_, (size_t)B * d, x_);
    }
  }
}


// EPI_TP_RESID (the O / down all-reduce in the GEMV epilogue, gemv_q8.h) when the comm provides the
// fused context
bool Engine::tp_fuse_gemv(GemvArgs a) {
  // batch 1 only, through the row-pair kernel (any K; a TP rank's O / down shares sit below the LDS
  // engine's size floor anyway); B = 2..4 keep separate all-reduce launches
  if (!tp_fuse_ || a.B != 1 || !a.act_q8 || a.force_v1 || a.nseg != 1) return false;  // (int8-activation kernel)
  const int qt0 = a.seg[0].qtype;
  if (!(qt0 == QT_Q4_K || qt0 == QT_Q5_K || qt0 == QT_Q6_K || qt0 == QT_Q4_0 || qt0 == QT_Q8_0)) return false;
  a.tp = tp_fuse_;
  a.kernel_sel = 1;
  a.tune_grid = 0;
  a.tune_u = 0;
  a.tune_ksplit = 0;
  a.grid_cap = tp_fuse_grid_;  // ranks sharing a GPU: every rank's workgroups resident together
  // (false: the row-pair kernel did not take it -- stage capacity within grid_cap, LDS plan -- and
  // nothing was launched; the caller runs the plain GEMV + all-reduce)
  return launch_gemv_tp_fused(a, stream_);
}

std::vector<int> Engine::tp_fuse_fits() {
  const CuScope cu_scope(cus_);  // (grids sized to this engine's CU mask)
  std::vector<int> out;
  if (!tp_fuse_) return out;
  HIP_CHECK(hipSetDevice(cfg_.device));
  const int d = cfg_.d_model, qd = cfg_.n_heads * cfg_.head_dim;
  for (int l = 0; l < cfg_.n_layers; ++l) {
    const LayerW& L = layers_[l];
    GemvArgs o = gemv_args({&L.wo}, d, qd, 1, attn_, qd, nullptr, x_, d, EPI_TP_RESID, l);
    GemvArgs f = gemv_args({&L.wdown}, d, cfg_.d_ff, 1, ff_, cfg_.d_ff, nullptr, x_, d, EPI_TP_RESID, l);
    o.dry = f.dry = 1;
    out.push_back(tp_fuse_gemv(o) ? 1 : 0);
    out.push_back(tp_fuse_gemv(f) ? 1 : 0);
  }
  return out;
}

// logits_[B][V] = rmsnorm(x) . output^T.  Vocab-parallel TP: this rank holds V/tp rows of
// output.weight, writes its column slice of every logits row, and the xGMI all-gather completes the
// rows on every rank, so the sampler and the grammar mask run identically everywhere -- 1/tp of
// the largest single matrix per GPU instead of a replica (Llama-3 70B: 128256 x 8192 Q6_K).
void Engine::lm_head(int B, const float* x, int ldx) {
  const int d = cfg_.d_model, V = cfg_.vocab_size;
  const bool vp = cfg_.vocab_parallel != 0;
  const int Vl = vp ? V / cfg_.tp_size : V;
  float* y = logits_ + (vp ? (size_t)cfg_.tp_rank * Vl : 0);
  if (dec_a16_ && ((dec_gemm_min_b_ > 0 && B >= dec_gemm_min_b_) || B > 8) && Vl % 64 == 0 &&
      gemm_supports(output_.w.qtype)) {
    const bool fused = nrm_lm_ && x == x_ && ldx == d;  // normalised by the last down GEMM
    nrm_lm_ = false;  // one use: a later lm_head (prefill) normalises for itself
    if (!fused) launch_rmsnorm_bf16(x, ldx, out_norm_, dec_a16_, d, B, d, cfg_.norm_eps, stream_);
    GemmQArgs g;
    std::memset(&g, 0, sizeof(g));
    g.A = dec_a16_; g.lda = d; g.M = B; g.K = d; g.nseg = 1; g.seg[0] = output_.w; g.N = Vl;
    g.C = y; g.ldc = V; g.epi = GEPI_STORE;
    if (fused) { g.A = dec_xn16_; g.nrm_in = lm_nrm_in_; g.nrm_parts = lm_nrm_parts_; g.nrm_eps = cfg_.norm_eps; }
    gemm(g);
  } else {
    gemv({&output_}, Vl, d, B, x, ldx, out_norm_, y, V, EPI_STORE, 0);
  }
  if (vp) {
    if (!allgather_) throw std::runtime_error("vocab-parallel engine without an all-gather hook");
    allgather_(allgather_ctx_, logits_, B, Vl, V, stream_);
  }
}

void Engine::enqueue_decode_step(int B) {
  enqueue_decode_forward(B);
  enqueue_sample(B);
}

void Engine::enqueue_decode_forward(int B) {
  const int d = cfg_.d_model;
  {
    StepPrep sp{d_pos_, d_slot_, d_bt_, kv_maxb_, rope_cs_, cfg_.head_dim / 2, d_step_kv_, d_step_rope_};
    launch_get_rows_step(tok_embd_.w, d_tokens_, B, x_, d, 1.f, sp, stream_);
  }
  static const bool step_prep = !(std::getenv("AIOS_STEP_PREP") && std::atoi(std::getenv("AIOS_STEP_PREP")) == 0);
  step_prep_on_ = step_prep && rope_cs_ != nullptr;
  nrm_lm_ = false;
  for (int l = 0; l < cfg_.n_layers; ++l) layer_decode(l, B);
  step_prep_on_ = false;
  lm_head(B, x_, d);
  nrm_lm_ = false;
}

void Engine::enqueue_sample(int B) {
  const int V = cfg_.vocab_size;
  SampleArgs s;
  std::memset(&s, 0, sizeof(s));
  s.logits = logits_; s.ldl = V; s.B = B; s.V = V;
  s.temperature = d_temp_; s.top_k = d_topk_;
  s.seed = sample_seed_;
  s.seed_dev = d_seed_;
  s.seeds = d_seeds_;
  s.tokens = d_tokens_; s.pos = d_pos_; s.seq_len = d_seqlen_;
  s.history = d_history_; s.hist_stride = cfg_.max_ctx + 1;
  s.advance = 1;
  s.mask = sample_mask_ ? d_mask_ : nullptr;
  s.top_p = d_topp_; s.ws = sample_ws_; s.ws_bytes = sample_ws_bytes_; s.counters = sample_cnt_;
  launch_sample(s, stream_);
}

bool Engine::gemm_prefill_ok(int T) const { return gm_ok_ && T >= gm_min_rows_; }

// Prefill through the matrix cores: per chunk of <= gm_rows_ tokens and per layer
//   RMSNorm -> bf16 | QKV GEMM (Q4_K/Q6_K dequant fused, one launch per format run) | RoPE + KV
//   write | causal flash attention (MFMA) -> bf16 | O GEMM (+= residual) | RMSNorm -> bf16 |
//   gate/up GEMM with the SwiGLU epilogue -> bf16 | down GEMM (+= residual)
// so every weight byte is dequantised once per chunk (not once per 8 rows as on the GEMV path).
// TP: the row-parallel O / down outputs go through the all-reduce hook into the residual.
void Engine::prefill_gemm(int slot, const std::vector<int>& tokens, int start_pos, bool want_logits) {
  TraceRange tr("aios.prefill_gemm");
  const int T = (int)tokens.size();
  const int d = cfg_.d_model, hd = cfg_.head_dim, H = cfg_.n_heads, Hkv = cfg_.n_kv_heads, ff = cfg_.d_ff;
  const int qd = H * hd, kvd = Hkv * hd, ldqkv = qd + 2 * kvd, V = cfg_.vocab_size;
  const bool tp = cfg_.tp_size > 1;
  std::vector<int> hp(gm_rows_), hs(gm_rows_, slot);
  // short chunks (n <= max_batch, the batched-decode GEMMs' shapes): the decode step's fusions --
  // RoPE + KV write in the QKV GEMM's epilogue and the split RMSNorm (the residual GEMMs write
  // bf16(x * g_next) + per-tile sums, the next GEMM scales its rows) -- 3 launches per layer fewer
  static const bool short_fuse = !(std::getenv("AIOS_PREFILL_SHORT_FUSE") && std::atoi(std::getenv("AIOS_PREFILL_SHORT_FUSE")) == 0);
  for (int r0 = 0; r0 < T; r0 += gm_rows_) {
    const int n = std::min(gm_rows_, T - r0);
    // (the fused epilogues are the ring GEMM's: chunks of <= 32 rows; longer chunks take the prefill
    // GEMM, kernels/gemm_pf.hip, with the plain epilogues)
    const bool sh = short_fuse && !tp && n <= 32;
    const bool fnp = sh && gm_nparts_ > 0;
    for (int i = 0; i < n; ++i) hp[i] = start_pos + r0 + i;
    HIP_CHECK(hipMemcpyAsync(gm_tokens_, tokens.data() + r0, n * 4, hipMemcpyHostToDevice, stream_));
    HIP_CHECK(hipMemcpyAsync(gm_pos_, hp.data(), n * 4, hipMemcpyHostToDevice, stream_));
    HIP_CHECK(hipMemcpyAsync(gm_slot_, hs.data(), n * 4, hipMemcpyHostToDevice, stream_));
    launch_get_rows(tok_embd_.w, gm_tokens_, n, gm_x_, d, 1.f, stream_);
    for (int l = 0; l < cfg_.n_layers; ++l) {
      const LayerW& L = layers_[l];
      bf16_t* kc = kv_layer(k_cache_, l);
      bf16_t* vc = kv_layer(v_cache_, l);
      // split-RMSNorm consumer / producer (as in layer_decode_gemm, on this chunk's rows)
      auto nrm_in = [&](GemmQArgs& g) {
        g.A = gm_xn16_; g.nrm_in = gm_npart_; g.nrm_parts = gm_nparts_; g.nrm_eps = cfg_.norm_eps;
      };
      auto nrm_out = [&](GemmQArgs& g, const float* g_next) {
        g.epi = GEPI_ACCUM_NORM; g.nrm_g = g_next; g.nrm_out16 = gm_xn16_; g.nrm_part = gm_npart_;
        g.nrm_parts = gm_nparts_;
      };
      if (!(fnp && l > 0)) launch_rmsnorm_bf16(gm_x_, d, L.attn_norm, gm_a16_, d, n, d, cfg_.norm_eps, stream_);
      GemmQArgs g;
      std::memset(&g, 0, sizeof(g));
      g.A = gm_a16_; g.lda = d; g.M = n; g.K = d;
      if (fnp && l > 0) nrm_in(g);
      g.nseg = 3;
      g.seg[0] = L.wq.w; g.seg[1] = L.wk.w; g.seg[2] = L.wv.w;
      g.seg_n0[0] = 0; g.seg_n0[1] = qd; g.seg_n0[2] = qd + kvd;
      g.N = ldqkv; g.C = gm_qkv_; g.ldc = ldqkv; g.epi = GEPI_STORE;
      // the RoPE / KV-cache epilogue: short chunks (ring / skinny GEMMs); the prefill GEMM's chunks
      // (>= 33 rows) only with AIOS_PREFILL_QKV_EPI=1 -- it needs S = 1 plans, and at 2048 tokens
      // the QKV GEMM then took 212.7 us against 115.7 (split-K) + 32 us of qkv_post (64 tokens:
      // 5.77 vs 4.6 ms per prompt), profiles/prefill_r5.txt
      const bool qepi_ok = !cfg_.qk_norm && !cfg_.rope_neox && !L.bqkv && rope_cs_ && !tp;
      bool qepi = false;
      if (qepi_ok) {
        GemmQArgs q = g;
        q.epi = GEPI_QKV; q.col0 = 0;
        q.head_dim = hd; q.q_dim = qd; q.kv_dim = kvd; q.n_kv_heads = Hkv; q.max_ctx = cfg_.max_ctx;
        q.rope_cs = rope_cs_; q.pos = gm_pos_; q.slot = gm_slot_; q.block_table = d_bt_;
        q.q_out = gm_q_; q.k_cache = kc; q.v_cache = vc;
        kv_write_args(q, l);
        static const int pf_qkv = [] { const char* e = std::getenv("AIOS_PREFILL_QKV_EPI"); return e ? std::atoi(e) : 0; }();
        qepi = sh || (pf_qkv && gemm_pf_serves(q));
        if (qepi) g = q;
      }
      gemm(g);
      if (!qepi) {
      QkvPostArgs p;
      p.qkv = gm_qkv_; p.ldqkv = ldqkv; p.T = n;
      p.n_heads = H; p.n_kv_heads = Hkv; p.head_dim = hd;
      p.bias = L.bqkv; p.q_norm = L.q_norm; p.k_norm = L.k_norm; p.eps = cfg_.norm_eps;
      p.rope_neox = cfg_.rope_neox; p.rope_base = cfg_.rope_theta; p.rope_cs = rope_cs_;
      p.pos = gm_pos_; p.slot = gm_slot_; p.q_out = gm_q_;
      p.k_cache = kc; p.v_cache = vc; p.max_ctx = cfg_.max_ctx; p.block_table = d_bt_;
      kv_write_args(p, l);
      launch_qkv_post(p, stream_);
      }
      AttnPrefillArgs at;
      at.q = gm_q_; at.k_cache = kc; at.v_cache = vc; at.block_table = d_bt_;
      kv_read_args(at, l);
      at.slot = slot; at.start = start_pos + r0; at.T = n;
      at.n_heads = H; at.n_kv_heads = Hkv; at.head_dim = hd; at.max_ctx = cfg_.max_ctx;
      at.scale = 1.f / std::sqrt((float)hd);
      at.out = gm_attn16_; at.ldo = qd;
      launch_attn_prefill(at, stream_);
      // O projection (+ residual)
      std::memset(&g, 0, sizeof(g));
      g.A = gm_attn16_; g.lda = qd; g.M = n; g.K = qd; g.nseg = 1; g.seg[0] = L.wo.w; g.N = d; g.ldc = d;
      if (tp) { g.C = gm_part_; g.epi = GEPI_STORE; } else { g.C = gm_x_; g.epi = GEPI_ACCUM; }
      if (fnp) nrm_out(g, L.ffn_norm);
      gemm(g);
      if (tp) allreduce(gm_part_, (size_t)n * d, gm_x_);
      // FFN
      if (!fnp) launch_rmsnorm_bf16(gm_x_, d, L.ffn_norm, gm_a16_, d, n, d, cfg_.norm_eps, stream_);
      std::memset(&g, 0, sizeof(g));
      g.A = gm_a16_; g.lda = d; g.M = n; g.K = d; g.nseg = 1; g.seg[0] = L.wgu.w; g.N = 2 * ff;
      g.C16 = gm_ff16_; g.ldc = ff; g.epi = GEPI_SWIGLU_BF16;
      if (fnp) nrm_in(g);
      gemm(g);
      std::memset(&g, 0, sizeof(g));
      g.A = gm_ff16_; g.lda = ff; g.M = n; g.K = ff; g.nseg = 1; g.seg[0] = L.wdown.w; g.N = d; g.ldc = d;
      if (tp) { g.C = gm_part_; g.epi = GEPI_STORE; } else { g.C = gm_x_; g.epi = GEPI_ACCUM; }
      if (fnp && l + 1 < cfg_.n_layers) nrm_out(g, layers_[l + 1].attn_norm);  // (lm_head normalises its row)
      gemm(g);
      if (tp) allreduce(gm_part_, (size_t)n * d, gm_x_);
    }
    if (r0 + n == T && want_logits) lm_head(1, gm_x_ + (size_t)(n - 1) * d, d);
  }
}

std::vector<float> Engine::prefill(int slot, const std::vector<int>& tokens, int start_pos, bool want_logits) {
  const CuScope cu_scope(cus_);  // (grids sized to this engine's CU mask)
  TraceRange tr("aios.prefill");
  if (!finalized_) throw std::runtime_error("engine not finalized");
  HIP_CHECK(hipSetDevice(cfg_.device));
  const int T = (int)tokens.size();
  if (T == 0) throw std::runtime_error("prefill: empty prompt");
  if (start_pos + T > cfg_.max_ctx) throw std::runtime_error("prefill: context overflow");
  if (slot < 0 || slot >= cfg_.max_slots) throw std::runtime_error("prefill: bad slot");
  for (int t : tokens)
    if (t < 0 || t >= cfg_.vocab_size) throw std::runtime_error("prefill: token id out of range");
  kv_prepare_write(slot, start_pos, start_pos + T);
  kv_sync(0);
  if (gemm_prefill_ok(T)) {
    prefill_gemm(slot, tokens, start_pos, want_logits);
    std::vector<float> out;
    if (want_logits) {
      out.resize(cfg_.vocab_size);
      HIP_CHECK(hipMemcpyAsync(out.data(), logits_, (size_t)cfg_.vocab_size * 4, hipMemcpyDeviceToHost, stream_));
    }
    HIP_CHECK(hipStreamSynchronize(stream_));
    return out;
  }
  const int d = cfg_.d_model, V = cfg_.vocab_size;
  const int R = prefill_rows_;
  // swap decode workspace pointers with the prefill ones for the duration of the call
  std::swap(x_, pf_x_); std::swap(q_, pf_q_); std::swap(qkv_, pf_qkv_); std::swap(attn_, pf_attn_);
  std::swap(ff_, pf_ff_); std::swap(opart_, pf_opart_); std::swap(ml_, pf_ml_);
  int* save_tok = d_tokens_; int* save_pos = d_pos_; int* save_sl = d_seqlen_; int* save_slot = d_slot_;
  std::vector<int> hp(R), hs(R), hsl(R);
  try {
    for (int r0 = 0; r0 < T; r0 += R) {
      const int n = std::min(R, T - r0);
      for (int i = 0; i < n; ++i) { hp[i] = start_pos + r0 + i; hsl[i] = hp[i] + 1; hs[i] = slot; }
      HIP_CHECK(hipMemcpyAsync(pf_tokens_, tokens.data() + r0, n * 4, hipMemcpyHostToDevice, stream_));
      HIP_CHECK(hipMemcpyAsync(pf_pos_, hp.data(), n * 4, hipMemcpyHostToDevice, stream_));
      HIP_CHECK(hipMemcpyAsync(pf_seqlen_, hsl.data(), n * 4, hipMemcpyHostToDevice, stream_));
      HIP_CHECK(hipMemcpyAsync(pf_slot_, hs.data(), n * 4, hipMemcpyHostToDevice, stream_));
      launch_get_rows(tok_embd_.w, pf_tokens_, n, x_, d, 1.f, stream_);
      float* xb = x_;
      float *qb = q_, *qkvb = qkv_, *ab = attn_, *fb = ff_;
      for (int l = 0; l < cfg_.n_layers; ++l) {
        // sub-batches of <= 8 rows through the GEMV path; attention over all n rows at once
        const int nsub = (n + 7) / 8;
        for (int sb = 0; sb < nsub; ++sb) {
          const int o = sb * 8, bn = std::min(8, n - o);
          x_ = xb + (size_t)o * d; q_ = qb + (size_t)o * cfg_.n_heads * cfg_.head_dim;
          qkv_ = qkvb + (size_t)o * (cfg_.n_heads + 2 * cfg_.n_kv_heads) * cfg_.head_dim;
          d_pos_ = pf_pos_ + o; d_slot_ = pf_slot_ + o; d_seqlen_ = pf_seqlen_ + o;
          // QKV only (layer_decode runs the whole block; split it by temporarily faking)
          const LayerW& L = layers_[l];
          const int hd = cfg_.head_dim, qd = cfg_.n_heads * hd, kvd = cfg_.n_kv_heads * hd;
          const bool fused_qkv = !cfg_.qk_norm && !cfg_.rope_neox;
          int row0 = 0;
          for (auto& grp : qkv_groups(L)) {
            int nn = 0;
            for (auto* m : grp) nn += m->w.rows;
            GemvArgs a;
            std::memset(&a, 0, sizeof(a));
  a.act_q8 = cfg_.act_q8;
            a.nseg = (int)grp.size();
            int r = 0;
            for (int s = 0; s < a.nseg; ++s) { a.seg[s] = grp[s]->w; a.seg_row0[s] = r; r += grp[s]->w.rows; }
            a.N = nn; a.K = d; a.B = bn; a.row_base = row0;
            a.x = x_; a.ldx = d; a.norm_w = L.attn_norm; a.eps = cfg_.norm_eps;
            if (fused_qkv) {
              a.epi = EPI_QKV; a.y = q_; a.ldy = qd; a.bias = L.bqkv;
              a.head_dim = hd; a.q_dim = qd; a.kv_dim = kvd; a.n_kv_heads = cfg_.n_kv_heads; a.max_ctx = cfg_.max_ctx;
              a.rope_neox = cfg_.rope_neox; a.rope_base = cfg_.rope_theta; a.rope_cs = rope_cs_;
              a.pos = d_pos_; a.slot = d_slot_;
              a.k_cache = kv_layer(k_cache_, l);
              a.v_cache = kv_layer(v_cache_, l);
              kv_write_args(a, l);
              a.block_table = d_bt_;
            } else {
              a.epi = EPI_STORE; a.y = qkv_; a.ldy = qd + 2 * kvd;
            }
            launch_gemv(a, stream_);
            row0 += nn;
          }
          if (!fused_qkv) {
            QkvPostArgs p;
            p.qkv = qkv_; p.ldqkv = qd + 2 * kvd; p.T = bn;
            p.n_heads = cfg_.n_heads; p.n_kv_heads = cfg_.n_kv_heads; p.head_dim = hd;
            p.q_norm = L.q_norm; p.k_norm = L.k_norm; p.eps = cfg_.norm_eps;
            p.rope_neox = cfg_.rope_neox; p.rope_base = cfg_.rope_theta; p.rope_cs = rope_cs_;
            p.pos = d_pos_; p.slot = d_slot_; p.q_out = q_;
            p.k_cache = kv_layer(k_cache_, l);
            p.v_cache = kv_layer(v_cache_, l);
            kv_write_args(p, l);
            p.max_ctx = cfg_.max_ctx;
            p.block_table = d_bt_;
            launch_qkv_post(p, stream_);
          }
        }
        // attention for all n rows (causal by per-row seq_len)
        {
          AttnDecodeArgs a;
          a.split = 0;
          a.q = qb;
          a.k_cache = kv_layer(k_cache_, l);
          a.v_cache = kv_layer(v_cache_, l);
          kv_read_args(a, l);
          a.seq_len = pf_seqlen_; a.slot = pf_slot_;
          a.block_table = d_bt_; a.bt_rows = 0;  // prefill rows: one slot, slot-indexed table
          a.B = n; a.n_heads = cfg_.n_heads; a.n_kv_heads = cfg_.n_kv_heads; a.head_dim = cfg_.head_dim;
          a.max_ctx = cfg_.max_ctx;
          a.n_chunks = n_chunks_;
          a.scale = 1.f / std::sqrt((float)cfg_.head_dim);
          a.o_part = opart_; a.ml = ml_; a.out = ab; a.counters = attn_cnt_;
          launch_attn_decode(a, stream_);
        }
        for (int sb = 0; sb < nsub; ++sb) {
          const int o = sb * 8, bn = std::min(8, n - o);
          const LayerW& L = layers_[l];
          const int qd = cfg_.n_heads * cfg_.head_dim;
          float* xr = xb + (size_t)o * d;
          if (cfg_.tp_size > 1) {
            gemv({&L.wo}, d, qd, bn, ab + (size_t)o * qd, qd, nullptr, fb + (size_t)o * d, d, EPI_STORE, l);
          } else {
            gemv({&L.wo}, d, qd, bn, ab + (size_t)o * qd, qd, nullptr, xr, d, EPI_RESID, l);
          }
        }
        if (cfg_.tp_size > 1) {
          allreduce(fb, (size_t)n * d, xb);
        }
        for (int sb = 0; sb < nsub; ++sb) {
          const int o = sb * 8, bn = std::min(8, n - o);
          const LayerW& L = layers_[l];
          gemv({&L.wgu}, 2 * cfg_.d_ff, d, bn, xb + (size_t)o * d, d, L.ffn_norm, fb + (size_t)o * cfg_.d_ff,
               cfg_.d_ff, EPI_SWIGLU, l);
        }
        for (int sb = 0; sb < nsub; ++sb) {
          const int o = sb * 8, bn = std::min(8, n - o);
          const LayerW& L = layers_[l];
          if (cfg_.tp_size > 1) {
            gemv({&L.wdown}, d, cfg_.d_ff, bn, fb + (size_t)o * cfg_.d_ff, cfg_.d_ff, nullptr, ab + (size_t)o * d,
                 d, EPI_STORE, l);
          } else {
            gemv({&L.wdown}, d, cfg_.d_ff, bn, fb + (size_t)o * cfg_.d_ff, cfg_.d_ff, nullptr, xb + (size_t)o * d,
                 d, EPI_RESID, l);
          }
        }
        if (cfg_.tp_size > 1) {
          allreduce(ab, (size_t)n * d, xb);
        }
      }
      x_ = xb; q_ = qb; qkv_ = qkvb; attn_ = ab; ff_ = fb;
      if (r0 + n == T && want_logits) lm_head(1, x_ + (size_t)(n - 1) * d, d);
    }
  } catch (...) {
    std::swap(x_, pf_x_); std::swap(q_, pf_q_); std::swap(qkv_, pf_qkv_); std::swap(attn_, pf_attn_);
    std::swap(ff_, pf_ff_); std::swap(opart_, pf_opart_); std::swap(ml_, pf_ml_);
    d_tokens_ = save_tok; d_pos_ = save_pos; d_seqlen_ = save_sl; d_slot_ = save_slot;
    throw;
  }
  std::swap(x_, pf_x_); std::swap(q_, pf_q_); std::swap(qkv_, pf_qkv_); std::swap(attn_, pf_attn_);
  std::swap(ff_, pf_ff_); std::swap(opart_, pf_opart_); std::swap(ml_, pf_ml_);
  d_tokens_ = save_tok; d_pos_ = save_pos; d_seqlen_ = save_sl; d_slot_ = save_slot;
  std::vector<float> out;
  if (want_logits) {
    out.resize(V);
    HIP_CHECK(hipMemcpyAsync(out.data(), logits_, (size_t)V * 4, hipMemcpyDeviceToHost, stream_));
  }
  HIP_CHECK(hipStreamSynchronize(stream_));
  return out;
}

std::vector<int> Engine::decode(const std::vector<int>& slots, const std::vector<int>& tokens,
                                const std::vector<int>& pos, const std::vector<float>& temperature,
                                const std::vector<int>& top_k, uint64_t seed, const std::vector<uint8_t>& mask,
                                const std::vector<float>& top_p, const std::vector<uint64_t>& seeds) {
  const CuScope cu_scope(cus_);  // (grids sized to this engine's CU mask)
  if (!finalized_) throw std::runtime_error("engine not finalized");
  HIP_CHECK(hipSetDevice(cfg_.device));
  const int B = (int)slots.size();
  if (!seeds.empty() && (int)seeds.size() != B) throw std::runtime_error("decode: seeds size mismatch");
  if (B < 1 || B > cfg_.max_batch) throw std::runtime_error("decode: batch out of range");
  if ((int)tokens.size() != B || (int)pos.size() != B) throw std::runtime_error("decode: size mismatch");
  std::vector<int> sl(B);
  for (int b = 0; b < B; ++b) {
    if (pos[b] < 0 || pos[b] >= cfg_.max_ctx) throw std::runtime_error("decode: position out of range");
    if (slots[b] < 0 || slots[b] >= cfg_.max_slots) throw std::runtime_error("decode: bad slot");
    if (tokens[b] < 0 || tokens[b] >= cfg_.vocab_size) throw std::runtime_error("decode: token out of range");
    sl[b] = pos[b] + 1;
  }
  row_slots_ = slots;
  row_pos_ = pos;
  const int Bm = cfg_.max_batch;
  const size_t mbytes = (size_t)B * ((cfg_.vocab_size + 7) / 8);
  sample_mask_ = !mask.empty();
  if (sample_mask_ && mask.size() != mbytes) throw std::runtime_error("decode: mask size mismatch");
  // one pinned staging block -> one async copy (layout: see finalize)
  *(uint64_t*)h_par_ = seed;  // device-resident seed: one captured graph per (B, masked) serves every request
  int* hs = (int*)(h_par_ + 8);
  int *ht = hs + Bm, *hp = ht + Bm, *hl = hp + Bm, *hk = hl + Bm;
  float* hT = (float*)(hk + Bm);
  float* hP = hT + Bm;
  for (int b = 0; b < B; ++b) {
    hs[b] = slots[b]; ht[b] = tokens[b]; hp[b] = pos[b]; hl[b] = sl[b];
    hk[b] = b < (int)top_k.size() ? top_k[b] : 0;
    hT[b] = b < (int)temperature.size() ? temperature[b] : 0.f;
    hP[b] = b < (int)top_p.size() ? top_p[b] : 1.f;
  }
  fill_row_seeds((uint64_t*)(h_par_ + ((char*)d_seeds_ - d_par_)), B, seed, seeds);
  size_t nbytes = (size_t)((char*)d_seeds_ - d_par_) + (size_t)Bm * 8;
  if (sample_mask_) {
    std::memcpy(h_par_ + par_mask_off_, mask.data(), mbytes);
    nbytes = par_mask_off_ + mbytes;
  }
  HIP_CHECK(hipMemcpyAsync(d_par_, h_par_, nbytes, hipMemcpyHostToDevice, stream_));
  decode_loop_run(B, 1, true);
  HIP_CHECK(hipMemcpyAsync(h_tok_out_, d_tokens_, B * 4, hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipStreamSynchronize(stream_));
  sample_mask_ = false;
  return std::vector<int>(h_tok_out_, h_tok_out_ + B);
}

std::vector<int> Engine::resample(int B, const std::vector<float>& temperature, const std::vector<int>& top_k,
                                  uint64_t seed, const std::vector<uint8_t>& mask, const std::vector<float>& top_p) {
  const CuScope cu_scope(cus_);  // (grids sized to this engine's CU mask)
  // re-run only the sampler on the logits of the last step (grammar fast path: the unmasked
  // sample was rejected on the host)
  HIP_CHECK(hipSetDevice(cfg_.device));
  std::vector<float> temps(B, 0.f);
  std::vector<int> tks(B, 0);
  for (int b = 0; b < B && b < (int)temperature.size(); ++b) temps[b] = temperature[b];
  for (int b = 0; b < B && b < (int)top_k.size(); ++b) tks[b] = top_k[b];
  HIP_CHECK(hipMemcpyAsync(d_temp_, temps.data(), B * 4, hipMemcpyHostToDevice, stream_));
  HIP_CHECK(hipMemcpyAsync(d_topk_, tks.data(), B * 4, hipMemcpyHostToDevice, stream_));
  std::vector<float> tps(B, 1.f);
  for (int b = 0; b < B && b < (int)top_p.size(); ++b) tps[b] = top_p[b];
  HIP_CHECK(hipMemcpyAsync(d_topp_, tps.data(), B * 4, hipMemcpyHostToDevice, stream_));
  HIP_CHECK(hipMemcpyAsync(d_seed_, &seed, 8, hipMemcpyHostToDevice, stream_));
  std::vector<uint64_t> hs(B);
  fill_row_seeds(hs.data(), B, seed, {});
  HIP_CHECK(hipMemcpyAsync(d_seeds_, hs.data(), (size_t)B * 8, hipMemcpyHostToDevice, stream_));
  const size_t mbytes = (size_t)B * ((cfg_.vocab_size + 7) / 8);
  if (!mask.empty()) {
    if (mask.size() != mbytes) throw std::runtime_error("resample: mask size mismatch");
    HIP_CHECK(hipMemcpyAsync(d_mask_, mask.data(), mbytes, hipMemcpyHostToDevice, stream_));
  }
  SampleArgs s;
  std::memset(&s, 0, sizeof(s));
  s.logits = logits_; s.ldl = cfg_.vocab_size; s.B = B; s.V = cfg_.vocab_size;
  s.temperature = d_temp_; s.top_k = d_topk_; s.seed_dev = d_seed_; s.seeds = d_seeds_;
  s.tokens = d_tokens_; s.pos = d_pos_; s.advance = 0;
  s.mask = mask.empty() ? nullptr : d_mask_;
  s.top_p = d_topp_; s.ws = sample_ws_; s.ws_bytes = sample_ws_bytes_; s.counters = sample_cnt_;
  // pos was advanced by the step: RNG key uses pos[b] (a different stream than the first sample)
  launch_sample(s, stream_);
  std::vector<int> out(B);
  HIP_CHECK(hipMemcpyAsync(out.data(), d_tokens_, B * 4, hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipStreamSynchronize(stream_));
  return out;
}

// rows without their own seed keep the shared seed decorrelated by row (the round-2 stream keyed
// (seed, row, pos)); rows with one (a request's own seed) sample independently of their row
void Engine::fill_row_seeds(uint64_t* hs, int B, uint64_t seed, const std::vector<uint64_t>& seeds) {
  for (int b = 0; b < B; ++b) hs[b] = seeds.empty() ? seed ^ (0x9E3779B97F4A7C15ULL * (uint64_t)(b + 1)) : seeds[b];
}

int Engine::sample_first(int pos, float temperature, int top_k, float top_p, uint64_t seed,
                         const std::vector<uint8_t>& mask) {
  const CuScope cu_scope(cus_);  // (grids sized to this engine's CU mask)
  if (!finalized_) throw std::runtime_error("engine not finalized");
  HIP_CHECK(hipSetDevice(cfg_.device));
  const size_t mbytes = (size_t)((cfg_.vocab_size + 7) / 8);
  if (!mask.empty() && mask.size() != mbytes) throw std::runtime_error("sample_first: mask size mismatch");
  // row 0 of the parameter block: the next decode() re-uploads every row it uses
  HIP_CHECK(hipMemcpyAsync(d_temp_, &temperature, 4, hipMemcpyHostToDevice, stream_));
  HIP_CHECK(hipMemcpyAsync(d_topk_, &top_k, 4, hipMemcpyHostToDevice, stream_));
  HIP_CHECK(hipMemcpyAsync(d_topp_, &top_p, 4, hipMemcpyHostToDevice, stream_));
  HIP_CHECK(hipMemcpyAsync(d_seeds_, &seed, 8, hipMemcpyHostToDevice, stream_));
  HIP_CHECK(hipMemcpyAsync(d_fpos_, &pos, 4, hipMemcpyHostToDevice, stream_));
  if (!mask.empty()) HIP_CHECK(hipMemcpyAsync(d_mask_, mask.data(), mbytes, hipMemcpyHostToDevice, stream_));
  SampleArgs s;
  std::memset(&s, 0, sizeof(s));
  s.logits = logits_; s.ldl = cfg_.vocab_size; s.B = 1; s.V = cfg_.vocab_size;
  s.temperature = d_temp_; s.top_k = d_topk_; s.seeds = d_seeds_;
  s.tokens = d_tokens_; s.pos = d_fpos_; s.advance = 0;
  s.mask = mask.empty() ? nullptr : d_mask_;
  s.top_p = d_topp_; s.ws = sample_ws_; s.ws_bytes = sample_ws_bytes_; s.counters = sample_cnt_;
  launch_sample(s, stream_);
  int out = 0;
  HIP_CHECK(hipMemcpyAsync(&out, d_tokens_, 4, hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipStreamSynchronize(stream_));
  return out;
}

std::vector<float> Engine::last_logits(int B) {
  std::vector<float> out((size_t)B * cfg_.vocab_size);
  HIP_CHECK(hipMemcpyAsync(out.data(), logits_, out.size() * 4, hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipStreamSynchronize(stream_));
  return out;
}

void Engine::decode_loop_prepare(const std::vector<int>& slots, const std::vector<int>& tokens,
                                 const std::vector<int>& pos) {
  const int B = (int)slots.size();
  if (B < 1 || B > cfg_.max_batch || (int)pos.size() != B || (int)tokens.size() != B)
    throw std::runtime_error("decode_loop_prepare: bad batch");
  std::vector<int> sl(B);
  for (int b = 0; b < B; ++b) sl[b] = pos[b] + 1;
  row_slots_ = slots;
  row_pos_ = pos;
  std::vector<float> temps(B, 0.f);
  std::vector<int> tks(B, 0);
  HIP_CHECK(hipMemcpyAsync(d_slot_, slots.data(), B * 4, hipMemcpyHostToDevice, stream_));
  HIP_CHECK(hipMemcpyAsync(d_tokens_, tokens.data(), B * 4, hipMemcpyHostToDevice, stream_));
  HIP_CHECK(hipMemcpyAsync(d_pos_, pos.data(), B * 4, hipMemcpyHostToDevice, stream_));
  HIP_CHECK(hipMemcpyAsync(d_seqlen_, sl.data(), B * 4, hipMemcpyHostToDevice, stream_));
  HIP_CHECK(hipMemcpyAsync(d_temp_, temps.data(), B * 4, hipMemcpyHostToDevice, stream_));
  HIP_CHECK(hipMemcpyAsync(d_topk_, tks.data(), B * 4, hipMemcpyHostToDevice, stream_));
  std::vector<float> ones(B, 1.f);
  HIP_CHECK(hipMemcpyAsync(d_topp_, ones.data(), B * 4, hipMemcpyHostToDevice, stream_));
  const uint64_t zero = 0;
  HIP_CHECK(hipMemcpyAsync(d_seed_, &zero, 8, hipMemcpyHostToDevice, stream_));
  std::vector<uint64_t> hs(B);
  fill_row_seeds(hs.data(), B, 0, {});
  HIP_CHECK(hipMemcpyAsync(d_seeds_, hs.data(), (size_t)B * 8, hipMemcpyHostToDevice, stream_));
  HIP_CHECK(hipStreamSynchronize(stream_));
  sample_seed_ = 0;
  sample_mask_ = false;
}

void Engine::decode_loop_run(int B, int n_steps, bool use_graph) {
  const CuScope cu_scope(cus_);  // (grids sized to this engine's CU mask)
  TraceRange tr(use_graph ? "aios.decode_graph_replay" : "aios.decode_eager");
  HIP_CHECK(hipSetDevice(cfg_.device));
  if ((int)row_slots_.size() < B) throw std::runtime_error("decode_loop_run: rows not prepared");
  // map (and un-share) the blocks the n steps will write, before any of them is enqueued
  for (int b = 0; b < B; ++b) {
    kv_prepare_write(row_slots_[b], row_pos_[b], std::min(row_pos_[b] + n_steps, cfg_.max_ctx));
    row_pos_[b] = std::min(row_pos_[b] + n_steps, cfg_.max_ctx);
  }
  kv_sync(B);
  if (!use_graph) {
    for (int i = 0; i < n_steps; ++i) enqueue_decode_step(B);
    return;
  }
  hipGraphExec_t ge = step_graph(B);
  for (int i = 0; i < n_steps; ++i) HIP_CHECK(hipGraphLaunch(ge, stream_));
}

// the captured decode step for (B, sample_mask_): captured once, replayed for every request --
// the kernels read tokens / positions / slots / sampling parameters from device arrays
hipGraphExec_t Engine::step_graph(int B) {
  const int key = B * 4 + (sample_mask_ ? 1 : 0);
  auto it = graphs_.find(key);
  if (it == graphs_.end()) {
    hipGraph_t g;
    HIP_CHECK(hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal));
    try {
      enqueue_decode_step(B);
    } catch (...) {
      hipStreamEndCapture(stream_, &g);
      throw;
    }
    HIP_CHECK(hipStreamEndCapture(stream_, &g));
    hipGraphExec_t ge;
    HIP_CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    HIP_CHECK(hipGraphDestroy(g));
    it = graphs_.emplace(key, ge).first;
  }
  return it->second;
}

// the forward of a decode step without its sampler (the pipelined decode's graph)
hipGraphExec_t Engine::forward_graph(int B) {
  const int key = B * 4 + 2;
  auto it = graphs_.find(key);
  if (it == graphs_.end()) {
    hipGraph_t g;
    HIP_CHECK(hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal));
    try {
      enqueue_decode_forward(B);
    } catch (...) {
      hipStreamEndCapture(stream_, &g);
      throw;
    }
    HIP_CHECK(hipStreamEndCapture(stream_, &g));
    hipGraphExec_t ge;
    HIP_CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    HIP_CHECK(hipGraphDestroy(g));
    it = graphs_.emplace(key, ge).first;
  }
  return it->second;
}

void Engine::decode_submit(const std::vector<int>& slots, const std::vector<int>& tokens, const std::vector<int>& pos,
                           const std::vector<float>& temperature, const std::vector<int>& top_k, uint64_t seed,
                           const std::vector<float>& top_p, const std::vector<uint64_t>& seeds) {
  const CuScope cu_scope(cus_);  // (grids sized to this engine's CU mask)
  if (!finalized_) throw std::runtime_error("engine not finalized");
  HIP_CHECK(hipSetDevice(cfg_.device));
  const int B = (int)slots.size();
  if (B < 1 || B > cfg_.max_batch) throw std::runtime_error("decode_submit: batch out of range");
  if ((int)pos.size() != B || (!tokens.empty() && (int)tokens.size() != B) || (!seeds.empty() && (int)seeds.size() != B))
    throw std::runtime_error("decode_submit: size mismatch");
  for (int b = 0; b < B; ++b) {
    if (pos[b] < 0 || pos[b] >= cfg_.max_ctx) throw std::runtime_error("decode_submit: position out of range");
    if (slots[b] < 0 || slots[b] >= cfg_.max_slots) throw std::runtime_error("decode_submit: bad slot");
    if (!tokens.empty() && (tokens[b] < 0 || tokens[b] >= cfg_.vocab_size))
      throw std::runtime_error("decode_submit: token out of range");
  }
  const int Bm = cfg_.max_batch;
  par_buf_ ^= 1;  // the other half: the previous submit's copy may not have run yet
  char* hpar = h_par_ + (size_t)par_buf_ * par_bytes_;
  *(uint64_t*)hpar = seed;
  int* hs = (int*)(hpar + 8);
  int *ht = hs + Bm, *hp = ht + Bm, *hl = hp + Bm, *hk = hl + Bm;
  float* hT = (float*)(hk + Bm);
  float* hP = hT + Bm;
  for (int b = 0; b < B; ++b) {
    hs[b] = slots[b]; hp[b] = pos[b]; hl[b] = pos[b] + 1;
    if (!tokens.empty()) ht[b] = tokens[b];
    hk[b] = b < (int)top_k.size() ? top_k[b] : 0;
    hT[b] = b < (int)temperature.size() ? temperature[b] : 0.f;
    hP[b] = b < (int)top_p.size() ? top_p[b] : 1.f;
  }
  const size_t seeds_off = (size_t)((char*)d_seeds_ - d_par_);
  fill_row_seeds((uint64_t*)(hpar + seeds_off), B, seed, seeds);
  const size_t tok_off = (size_t)((char*)d_tokens_ - d_par_), end = seeds_off + (size_t)Bm * 8;
  if (tokens.empty()) {  // every row array but the tokens the previous sampler left on the device
    const size_t after = tok_off + (size_t)Bm * 4;
    HIP_CHECK(hipMemcpyAsync(d_par_, hpar, tok_off, hipMemcpyHostToDevice, stream_));
    HIP_CHECK(hipMemcpyAsync(d_par_ + after, hpar + after, end - after, hipMemcpyHostToDevice, stream_));
  } else {
    HIP_CHECK(hipMemcpyAsync(d_par_, hpar, end, hipMemcpyHostToDevice, stream_));
  }
  row_slots_ = slots;
  row_pos_ = pos;
  for (int b = 0; b < B; ++b) {
    kv_prepare_write(slots[b], pos[b], pos[b] + 1);
    row_pos_[b] = pos[b] + 1;
  }
  kv_sync(B);
  HIP_CHECK(hipGraphLaunch(forward_graph(B), stream_));
  pipe_B_ = B;
}

void Engine::decode_sample(const std::vector<uint8_t>& mask) {
  const CuScope cu_scope(cus_);  // (grids sized to this engine's CU mask)
  const int B = pipe_B_;
  if (B < 1) throw std::runtime_error("decode_sample: no submitted step");
  HIP_CHECK(hipSetDevice(cfg_.device));
  const size_t mbytes = (size_t)B * ((cfg_.vocab_size + 7) / 8);
  if (!mask.empty()) {
    if (mask.size() != mbytes) throw std::runtime_error("decode_sample: mask size mismatch");
    // (one pinned buffer: the previous mask's copy ran before the sampler whose token the host
    // already collected)
    std::memcpy(h_mask_, mask.data(), mbytes);
    HIP_CHECK(hipMemcpyAsync(d_mask_, h_mask_, mbytes, hipMemcpyHostToDevice, stream_));
  }
  sample_mask_ = !mask.empty();
  enqueue_sample(B);
  sample_mask_ = false;
  HIP_CHECK(hipMemcpyAsync(h_tok_out_, d_tokens_, B * 4, hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipEventRecord(pipe_ev_, stream_));
}

std::vector<int> Engine::decode_collect() {
  const int B = pipe_B_;
  if (B < 1) throw std::runtime_error("decode_collect: no sampled step");
  HIP_CHECK(hipEventSynchronize(pipe_ev_));
  return std::vector<int>(h_tok_out_, h_tok_out_ + B);
}

// capture (without running) the decode-step graphs of every batch size up to max_b, masked and
// unmasked, so a serving scheduler whose batch grows and shrinks never stalls a step on a capture
// (a 160-launch capture + instantiate costs milliseconds); returns the graphs held
int Engine::capture_graphs(int max_b) {
  const CuScope cu_scope(cus_);  // (grids sized to this engine's CU mask)
  if (!finalized_) throw std::runtime_error("engine not finalized");
  HIP_CHECK(hipSetDevice(cfg_.device));
  const bool saved = sample_mask_;
  for (int B = 1; B <= std::min(max_b, cfg_.max_batch); ++B)
    for (int m = 0; m < 2; ++m) {
      sample_mask_ = m != 0;
      step_graph(B);
      if (m == 0) forward_graph(B);  // (the pipelined decode's forward)
    }
  sample_mask_ = saved;
  return (int)graphs_.size();
}

std::vector<int> Engine::decode_loop_history(int B, int from_pos, int n) {
  std::vector<int> out((size_t)B * n);
  for (int b = 0; b < B; ++b)
    HIP_CHECK(hipMemcpyAsync(out.data() + (size_t)b * n, d_history_ + (size_t)b * (cfg_.max_ctx + 1) + from_pos,
                             n * 4, hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipStreamSynchronize(stream_));
  return out;
}

void Engine::synchronize() {
  HIP_CHECK(hipStreamSynchronize(stream_));
}

void Engine::set_kv_scales(const std::vector<float>& s) {
  if (s.size() != (size_t)2 * cfg_.n_layers) throw std::runtime_error("set_kv_scales: need 2 x n_layers values");
  for (float v : s)
    if (!(v > 0.f) || !std::isfinite(v)) throw std::runtime_error("set_kv_scales: scales must be positive");
  if (finalized_) HIP_CHECK(hipStreamSynchronize(stream_));  // (no replay of the old graphs in flight)
  kv_scale_ = s;
  reset_graphs();
}

void Engine::reset_graphs() {
  for (auto& kv : graphs_) hipGraphExecDestroy(kv.second);
  graphs_.clear();
}

// ---- paged KV ----------------------------------------------------------------------------------
int Engine::kv_alloc() {
  if (free_blocks_.empty()) throw std::runtime_error("paged KV: pool exhausted");  // cannot happen, see finalize
  const int b = free_blocks_.back();
  free_blocks_.pop_back();
  refcnt_[b] = 1;
  return b;
}

void Engine::kv_unref(int blk) {
  if (blk < 0) return;
  if (--refcnt_[blk] == 0) free_blocks_.push_back(blk);
}

// one block of every layer's K and V pool: [n_kv_heads][KV_BLOCK][hd] contiguous
void Engine::kv_copy_block(int src, int dst) {
  const size_t blk = (size_t)cfg_.n_kv_heads * KV_BLOCK * cfg_.head_dim * kv_es_;  // bytes
  for (int l = 0; l < cfg_.n_layers; ++l)
    for (bf16_t* base : {k_cache_, v_cache_}) {
      char* lb = (char*)kv_layer(base, l);
      HIP_CHECK(hipMemcpyAsync(lb + (size_t)dst * blk, lb + (size_t)src * blk, blk, hipMemcpyDeviceToDevice, stream_));
    }
}

void Engine::kv_prepare_write(int slot, int from, int to) {
  if (slot < 0 || slot >= cfg_.max_slots) throw std::runtime_error("paged KV: bad slot");
  if (to <= from) return;
  int* row = bt_.data() + (size_t)slot * kv_maxb_;
  for (int j = from / KV_BLOCK; j <= (to - 1) / KV_BLOCK && j < kv_maxb_; ++j) {
    if (row[j] < 0) {
      row[j] = kv_alloc();
      bt_dirty_ = true;
    } else if (refcnt_[row[j]] > 1) {  // shared prefix block about to be written: un-share
      const int nb = kv_alloc();
      kv_copy_block(row[j], nb);
      kv_unref(row[j]);
      row[j] = nb;
      bt_dirty_ = true;
    }
  }
}

// Upload the slot table (when dirty) and the row table of decode rows 0..B-1 (when it changed).
// Blocking uploads with the stream drained first: the captured decode graph reads the tables in
// place, and a table changes only every KV_BLOCK tokens of a sequence or when rows change.
void Engine::kv_sync(int B) {
  bool rows_changed = false;
  std::vector<int> rows((size_t)B * kv_maxb_);
  for (int b = 0; b < B; ++b)
    for (int j = 0; j < kv_maxb_; ++j) {
      const int v = bt_[(size_t)row_slots_[b] * kv_maxb_ + j];
      rows[(size_t)b * kv_maxb_ + j] = v < 0 ? kv_nblocks_ : v;
    }
  if (B > 0 && std::memcmp(rows.data(), row_bt_host_.data(), rows.size() * 4) != 0) rows_changed = true;
  if (!bt_dirty_ && !rows_changed) return;
  HIP_CHECK(hipStreamSynchronize(stream_));
  if (bt_dirty_) {
    std::vector<int> dev(bt_.size());
    for (size_t i = 0; i < bt_.size(); ++i) dev[i] = bt_[i] < 0 ? kv_nblocks_ : bt_[i];
    // (on the engine's stream, not the null stream: a co-resident tier's CU-masked stream is a
    // blocking stream, and a null-stream copy would wait for the other tier's queued steps)
    HIP_CHECK(hipMemcpyAsync(d_bt_, dev.data(), dev.size() * 4, hipMemcpyHostToDevice, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
    bt_dirty_ = false;
  }
  if (rows_changed) {
    std::copy(rows.begin(), rows.end(), row_bt_host_.begin());
    HIP_CHECK(hipMemcpyAsync(d_row_bt_, rows.data(), rows.size() * 4, hipMemcpyHostToDevice, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
  }
}

void Engine::copy_slot(int src, int dst, int n) {
  const CuScope cu_scope(cus_);  // (grids sized to this engine's CU mask)
  if (!finalized_) throw std::runtime_error("engine not finalized");
  if (src < 0 || src >= cfg_.max_slots || dst < 0 || dst >= cfg_.max_slots) throw std::runtime_error("copy_slot: bad slot");
  if (src == dst) return;
  HIP_CHECK(hipSetDevice(cfg_.device));
  n = std::min(n, cfg_.max_ctx);
  int* s = bt_.data() + (size_t)src * kv_maxb_;
  int* d = bt_.data() + (size_t)dst * kv_maxb_;
  for (int j = 0; j < kv_maxb_; ++j) {  // dst's old content is dropped
    kv_unref(d[j]);
    d[j] = -1;
  }
  const int full = std::max(n, 0) / KV_BLOCK;
  for (int j = 0; j < full; ++j) {
    d[j] = s[j];
    if (d[j] >= 0) ++refcnt_[d[j]];
  }
  if (n > 0 && n % KV_BLOCK && s[full] >= 0) {  // the partial block: private copy
    d[full] = kv_alloc();
    kv_copy_block(s[full], d[full]);
  }
  bt_dirty_ = true;
  kv_sync(0);
  HIP_CHECK(hipStreamSynchronize(stream_));
}

void Engine::release_slot(int slot) {
  if (slot < 0 || slot >= cfg_.max_slots) throw std::runtime_error("release_slot: bad slot");
  int* row = bt_.data() + (size_t)slot * kv_maxb_;
  for (int j = 0; j < kv_maxb_; ++j) {
    if (row[j] >= 0) bt_dirty_ = true;
    kv_unref(row[j]);
    row[j] = -1;
  }
}

std::vector<int> Engine::block_table(int slot) const {
  if (slot < 0 || slot >= cfg_.max_slots) throw std::runtime_error("block_table: bad slot");
  return std::vector<int>(bt_.begin() + (size_t)slot * kv_maxb_, bt_.begin() + (size_t)(slot + 1) * kv_maxb_);
}

}  // namespace aios
