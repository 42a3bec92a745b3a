// BF16 weights on the batch 1..4 LDS-DMA decode engine (BASELINE config 2: TinyLlama-1.1B BF16, the
// operational tier); included by gemv_impl.h after gemv_lds.h, whose ring protocol it shares.
//
// Round 5 left 16-bit weights on the round-1 persistent register GEMV (fp32 x in LDS, two work items
// in flight per wave: 852 tok/s = 1.8 TB/s for TinyLlama BF16).  Here the weight stream is the
// engine's: per CU one 1024-thread workgroup, waves 14-15 copy whole 1 KB groups (512 weights of one
// row -- a BF16 row is K * 2 contiguous bytes, so group g of a segment sits at p0 + g * 1024) HBM ->
// LDS with global_load_lds_dwordx4 into a ring of R slots of 28 groups; waves 0-13 stage x ONCE as
// bf16 (times the RMSNorm weight; the 1 / rms scalar is applied to the row sums) and dot each slot's
// groups with v_dot2_f32_bf16: a 32-lane half-wave takes one group, a lane two contiguous 16-B pieces
// (cols p*8 and 256 + p*8 of the group: conflict-free ds_read_b128 of weights and x), 8 dot2 per
// staged x row.  No dequantisation: the dot work per byte is a third of the Q4_K engine's.
//
// Epilogues as the quantised engine (RMSNorm scale, QKV RoPE + paged KV write, SwiGLU with the bf16
// hand-off to the down projection, residual); EPI_TP_RESID stays with the row kernels.
#pragma once
// (included inside namespace aios by gemv_impl.h)

// slot geometry: GPW groups per consumer wave per step (2: one per half-wave, 28 KB slots; 1: one
// per wave, 14 KB slots -- a smaller prologue burst, a deeper ring for the same LDS)
template <int GPW>
struct LbSlot {
  static constexpr int NGS = LG_NG * GPW;   // groups per slot
  static constexpr int BYTES = NGS * 1024;
  static constexpr int PL = NGS / LG_NL;    // DMA instructions per loader wave per slot
  static_assert(NGS % LG_NL == 0, "every loader issues the same count per slot");
};

typedef __bf16 lb_bf16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float lb_dot2(uint32_t w, uint32_t x, float c) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(lb_bf16x2, w), __builtin_bit_cast(lb_bf16x2, x), c,
                                         false);
}
__device__ __forceinline__ float lb_dot8(const uint4& w, const uint4& x, float c) {
  c = lb_dot2(w.x, x.x, c);
  c = lb_dot2(w.y, x.y, c);
  c = lb_dot2(w.z, x.z, c);
  return lb_dot2(w.w, x.w, c);
}
__device__ __forceinline__ uint32_t lb_pk(float a, float b) {
  return (uint32_t)f32_to_bf16(a) | ((uint32_t)f32_to_bf16(b) << 16);
}

// slot s of this workgroup's groups [gw0, gw0 + ngroups) -> ring buffer dst.  Instruction i copies
// group gw0 + s * NGS + i (clamped to the last one: the tail slot re-reads it into unused space);
// loader lw issues i = lw, lw + NL, ...  The group index is wave-uniform, so the segment select is
// scalar and the only per-lane address term is lane * 16.
template <int GPW>
__device__ __forceinline__ void lb_dma_slot(const GemvArgs& a, uint8_t* dst, int s, int lw, int gw0, int glast,
                                            int nit) {
  constexpr int LB_NGS = LbSlot<GPW>::NGS, LB_PL = LbSlot<GPW>::PL;
  const int lane = threadIdx.x & 63;
  const int G1 = a.nseg > 1 ? a.seg_row0[1] * nit : 0x7fffffff;
  const int G2 = a.nseg > 2 ? a.seg_row0[2] * nit : 0x7fffffff;
  const uint64_t b0 = (uint64_t)sgpr_ptr(a.seg[0].p0);
  const uint64_t b1 = (uint64_t)sgpr_ptr(a.seg[1].p0) - (uint64_t)(a.nseg > 1 ? G1 : 0) * 1024;
  const uint64_t b2 = (uint64_t)sgpr_ptr(a.seg[2].p0) - (uint64_t)(a.nseg > 2 ? G2 : 0) * 1024;
#pragma unroll
  for (int k = 0; k < LB_PL; ++k) {
    const int i = lw + k * LG_NL;
    const int g = min(gw0 + s * LB_NGS + i, glast);
    const uint64_t base = g >= G2 ? b2 : (g >= G1 ? b1 : b0);
    const uint8_t* src = (const uint8_t*)(base + (uint64_t)g * 1024 + lane * 16);
    __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(dst + i * 1024), 16,
                                     0, 2 /* nt */);
  }
}

// x (B rows, fp32 or the bf16 SwiGLU hand-off) times the norm weight -> bf16 in LDS; per-wave sums of
// squares of the raw x -> red[wave][b].  Staging threads: the consumer waves.
template <int B>
__device__ __forceinline__ void lb_stage(const GemvArgs& a, uint16_t* xs, float* red) {
  const int tid = threadIdx.x, nthr = LG_NG * 64;
  const int noct = a.K >> 3, total = a.B * noct;
  float ssq[B];
#pragma unroll
  for (int b = 0; b < B; ++b) ssq[b] = 0.f;
  for (int t = tid; t < total; t += nthr) {
    const int b = t / noct, o = t - b * noct;
    float v[8];
    if (a.x16) {
      const uint4 u = *(const uint4*)(a.x16 + (size_t)b * a.ldx + 8 * o);
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) { v[2 * i] = __uint_as_float(w[i] << 16); v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u); }
    } else {
      const float4 f0 = *(const float4*)(a.x + (size_t)b * a.ldx + 8 * o);
      const float4 f1 = *(const float4*)(a.x + (size_t)b * a.ldx + 8 * o + 4);
      v[0] = f0.x; v[1] = f0.y; v[2] = f0.z; v[3] = f0.w; v[4] = f1.x; v[5] = f1.y; v[6] = f1.z; v[7] = f1.w;
    }
    if (a.norm_w) {
      float s2 = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) s2 = fmaf(v[i], v[i], s2);
#pragma unroll
      for (int bb = 0; bb < B; ++bb)
        if (bb == b) ssq[bb] += s2;
      const float4 g0 = *(const float4*)(a.norm_w + 8 * o), g1 = *(const float4*)(a.norm_w + 8 * o + 4);
      v[0] *= g0.x; v[1] *= g0.y; v[2] *= g0.z; v[3] *= g0.w; v[4] *= g1.x; v[5] *= g1.y; v[6] *= g1.z; v[7] *= g1.w;
    }
    *(uint4*)(xs + (size_t)b * a.K + 8 * o) = make_uint4(lb_pk(v[0], v[1]), lb_pk(v[2], v[3]), lb_pk(v[4], v[5]),
                                                         lb_pk(v[6], v[7]));
  }
  if (a.norm_w) {
    const int wave = tid >> 6, lane = tid & 63;
#pragma unroll
    for (int b = 0; b < B; ++b) {
      const float s = wave_sum(ssq[b]);
      if (lane == 0) red[wave * B + b] = s;
    }
  }
}

template <int B, int R, int GPW = 2>
__global__ void __launch_bounds__(LG_THREADS) gemv_lds16(GemvArgs a, CuPlan pl) {
  kernarg_warm<sizeof(GemvArgs) + sizeof(CuPlan)>();
  constexpr int LB_NGS = LbSlot<GPW>::NGS, LB_SLOT = LbSlot<GPW>::BYTES, LB_PL = LbSlot<GPW>::PL, LB_GPW = GPW;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int nit = a.K >> 9;  // 1 KB groups per row
  const int npairs = a.N >> 1;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = blockIdx.x;
  const int pb = (int)((long)g * npairs / (int)gridDim.x), pe = (int)((long)(g + 1) * npairs / (int)gridDim.x);
  if (pb >= pe) return;  // whole workgroup, before any barrier
  const int r0 = 2 * pb, nrows = 2 * (pe - pb);
  const int ngroups = nrows * nit;
  const int T = (ngroups + LB_NGS - 1) / LB_NGS;

  // ---- LDS: red[64] | rowacc[B][racc_n] | x (bf16) [B][K] | ring [R][28 KB]
  float* red = smem;
  float* rowacc = smem + 64;
  uint16_t* xs = (uint16_t*)(rowacc + B * pl.racc_n);
  const int ring_off = (int)(((const uint8_t*)(xs + (size_t)B * a.K) - (const uint8_t*)smem + 255) & ~255);
  uint8_t* ring = (uint8_t*)smem + ring_off;
  for (int i = threadIdx.x; i < B * pl.racc_n; i += LG_THREADS) rowacc[i] = 0.f;
  if (threadIdx.x < 64) red[threadIdx.x] = 0.f;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

  if (wave >= LG_NG) {
    // ---- loaders: R - 1 slots ahead, one counted wait + raw barrier per step (gemv_lds.h protocol)
    const int lw = wave - LG_NG;
    const int gw0 = r0 * nit, glast = gw0 + ngroups - 1;
    const int npro = min(T, R - 1);
    for (int s = 0; s < npro; ++s) lb_dma_slot<GPW>(a, ring + (size_t)s * LB_SLOT, s, lw, gw0, glast, nit);
    if (npro == R - 1) lg_vmcnt<(R - 2) * LB_PL>();
    else lg_vmcnt<0>();
    lg_barrier();  // B1: slot 0 landed, x staged
    for (int t = 0; t < T; ++t) {
      if (t + R - 1 < T) {
        lb_dma_slot<GPW>(a, ring + (size_t)((t + R - 1) % R) * LB_SLOT, t + R - 1, lw, gw0, glast, nit);
        lg_vmcnt<(R - 2) * LB_PL>();  // slot t + 1 landed
      } else {
        lg_vmcnt<0>();
      }
      lg_barrier();
    }
    lg_barrier();  // final
    return;
  }

  // ---- consumers
  float2 rope = make_float2(1.f, 0.f);
  int pos0 = 0, kv_blk0 = 0;
  if (B == 1 && a.epi == EPI_QKV && wave == 0) {
    pos0 = a.pos[0];
    kv_blk0 = kv_block(a.block_table, a.max_ctx / KV_BLOCK, a.slot ? a.slot[0] : 0, pos0);
    if (a.rope_cs) {
      int part, head, lrr;
      qkv_part(a, a.row_base + r0 + 2 * lane, part, head, lrr);
      rope = a.rope_cs[(size_t)pos0 * (a.head_dim >> 1) + (part < 2 ? (lrr >> 1) : 0)];
    }
  }
  lb_stage<B>(a, xs, red);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  lg_barrier();  // B1
  if constexpr (GPW == 1) {
    // one group per wave: lane p takes 16 B (cols p * 8 of the group's 512), a full-wave row sum
    const int kk = wave;
    const int dq = LB_NGS / nit, dr = LB_NGS - dq * nit;
    int row = kk / nit, it = kk - row * nit;
    for (int t = 0; t < T; ++t) {
      const int gg = t * LB_NGS + kk;
      if (gg < ngroups) {
        const uint4 w0 = *(const uint4*)(ring + (size_t)(t % R) * LB_SLOT + kk * 1024 + lane * 16);
        const int col = it * 512 + lane * 8;
        float v[B];
#pragma unroll
        for (int b = 0; b < B; ++b) v[b] = lb_dot8(w0, *(const uint4*)(xs + (size_t)b * a.K + col), 0.f);
        if constexpr (B == 1) {
          const float r = cu_wave_sum(v[0]);
          if (lane == 0) __hip_atomic_fetch_add(&rowacc[row], r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else {
          float r = lg_half_sum_rows<B>(v, lane & 31);
          const auto h = __builtin_amdgcn_permlane32_swap(__float_as_uint(r), __float_as_uint(r), false, false);
          r = __uint_as_float(h[0]) + __uint_as_float(h[1]);  // both 32-lane halves
          const int rb = lg_half_row<B>(lane & 31);
          if (lane < (B > 2 ? 4 : 2) && rb < B)
            __hip_atomic_fetch_add(&rowacc[rb * pl.racc_n + row], r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
      row += dq;
      it += dr;
      if (it >= nit) { it -= nit; ++row; }
      lg_barrier();
    }
  } else {
    const int half = lane >> 5, p = lane & 31;
    const int kk = wave * LB_GPW + half;  // this half-wave's group within a slot
    // (row, column group) of group t * NGS + kk, advanced by NGS per step without a division
    const int dq = LB_NGS / nit, dr = LB_NGS - dq * nit;
    int row = kk / nit, it = kk - row * nit;
    for (int t = 0; t < T; ++t) {
      const int gg = t * LB_NGS + kk;
      if (t * LB_NGS + wave * LB_GPW < ngroups) {
        const uint8_t* gp = ring + (size_t)(t % R) * LB_SLOT + kk * 1024;
        const uint4 w0 = *(const uint4*)(gp + p * 16);
        const uint4 w1 = *(const uint4*)(gp + 512 + p * 16);
        const bool ok = gg < ngroups;
        const int col = it * 512 + p * 8;
        float v[B];
#pragma unroll
        for (int b = 0; b < B; ++b) {
          const uint16_t* xb = xs + (size_t)b * a.K + col;
          const uint4 x0 = *(const uint4*)xb;
          const uint4 x1 = *(const uint4*)(xb + 256);
          v[b] = ok ? lb_dot8(w1, x1, lb_dot8(w0, x0, 0.f)) : 0.f;
        }
        if constexpr (B == 1) {
          const float r = cu_half_sum(v[0]);
          if (p == 0 && ok)
            __hip_atomic_fetch_add(&rowacc[row], r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else {
          const float r = lg_half_sum_rows<B>(v, p);
          const int rb = lg_half_row<B>(p);
          if (p < (B > 2 ? 4 : 2) && rb < B && ok)  // one LDS atomic instruction for all B rows
            __hip_atomic_fetch_add(&rowacc[rb * pl.racc_n + row], r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
      row += dq;
      it += dr;
      if (it >= nit) { it -= nit; ++row; }
      lg_barrier();
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  lg_barrier();  // final: every row sum is in rowacc
  if (wave != 0) return;

  if constexpr (B > 1) {
    float sb[B];
#pragma unroll
    for (int b = 0; b < B; ++b) {
      sb[b] = 1.f;
      if (a.norm_w) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < LG_NG; ++w) t += red[w * B + b];
        sb[b] = rsqrtf(t / (float)a.K + a.eps);
      }
    }
    const int npl = nrows >> 1;
    for (int i = lane; i < a.B * npl; i += 64) {
      const int b = i / npl, p = i - b * npl;
      float s_ = sb[0];
#pragma unroll
      for (int bb = 1; bb < B; ++bb)
        if (b == bb) s_ = sb[bb];
      gemv_epilogue(a, a.row_base + r0 + 2 * p, b, rowacc[b * pl.racc_n + 2 * p] * s_,
                    rowacc[b * pl.racc_n + 2 * p + 1] * s_);
    }
    return;
  } else {
    float s = 1.f;
    if (a.norm_w) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < LG_NG; ++w) t += red[w];
      s = rsqrtf(t / (float)a.K + a.eps);
    }
    for (int p = lane; 2 * p < nrows; p += 64) {
      const int grow = a.row_base + r0 + 2 * p;
      const float v0 = rowacc[2 * p] * s, v1 = rowacc[2 * p + 1] * s;
      if (a.epi == EPI_QKV) {
        float2 t = rope;
        if (p >= 64 || !a.rope_cs) {
          int part, head, lrr;
          qkv_part(a, grow, part, head, lrr);
          const int pp = lrr >> 1;
          if (a.rope_cs) {
            t = a.rope_cs[(size_t)pos0 * (a.head_dim >> 1) + pp];
          } else {
            float sn, cs;
            sincosf((float)pos0 * powf(a.rope_base, -2.f * (float)pp / (float)a.head_dim), &sn, &cs);
            t = make_float2(cs, sn);
          }
        }
        cu_qkv_epilogue(a, grow, v0, v1, t, pos0, kv_blk0);
      } else {
        gemv_epilogue1(a, grow, v0, v1);
      }
    }
  }
}

template <int B, int R, int GPW = 2>
size_t lb_lds_bytes(const GemvArgs& a, const CuPlan& pl) {
  const size_t head = (64 + (size_t)B * pl.racc_n) * 4 + (size_t)B * a.K * 2;
  return (head + 255) / 256 * 256 + (size_t)R * LbSlot<GPW>::BYTES;
}

// The BF16 engine for B = 1..4, or false (shape / epilogue outside it: the register kernels run).
// dry = true: only whether it would serve these args.
inline bool launch_gemv_lds16(const GemvArgs& a, hipStream_t st, bool dry = false) {
  // AIOS_GEMV_BF16_LDS=0: the round-1 persistent register GEMV instead (A/B runs)
  static const bool on = !(std::getenv("AIOS_GEMV_BF16_LDS") && std::atoi(std::getenv("AIOS_GEMV_BF16_LDS")) == 0);
  if (!on || a.B < 1 || a.B > 4 || a.K % 512 || a.N % 2 || a.epi == EPI_TP_RESID || a.tune_dbg ||
      (a.kernel_sel != 0 && a.kernel_sel != 3))
    return false;
  for (int s = 0; s < a.nseg; ++s)
    if (a.seg[s].qtype != QT_BF16 || a.seg[s].cols != a.K || (s > 0 && a.seg_row0[s] % 2)) return false;
  const int npairs = a.N / 2;
  const int G = std::min(a.tune_grid > 0 ? a.tune_grid : device_cu_count(), npairs);
  const CuPlan pl{G, npairs, (2 * ((npairs + G - 1) / G) + 3) & ~3};
  constexpr size_t LDS_MAX = 160 * 1024;
  // R = 3 (two 28 KB slots in flight per CU, the quantised engine's batch-1 depth), R = 2 where the
  // staged x rows leave no room (long K at B = 3..4)
  // AIOS_LB_CFG (batch 1 only): slot geometry x ring depth -- 23 = 28 KB slots x 3 (default),
  // 24 = 28 KB x 4, 14 = 14 KB x 4, 16 = 14 KB x 6 (profiles/decode_tinyllama_bf16_rocprof_r6.txt)
  static const int cfg = [] {
    const char* e = std::getenv("AIOS_LB_CFG");
    return e ? std::atoi(e) : 23;
  }();
  if (a.B == 1 && cfg != 23) {
    auto b1 = [&](auto gp, auto rr) -> bool {
      constexpr int GP = decltype(gp)::value, RR = decltype(rr)::value;
      const size_t lds = lb_lds_bytes<1, RR, GP>(a, pl);
      if (lds > LDS_MAX) return false;
      if (!dry) hipLaunchKernelGGL((gemv_lds16<1, RR, GP>), dim3(G), dim3(LG_THREADS), lds, st, a, pl);
      return true;
    };
    using I = std::integral_constant<int, 1>;
    using II = std::integral_constant<int, 2>;
    if (cfg == 24 && b1(II{}, std::integral_constant<int, 4>{})) return true;
    if (cfg == 14 && b1(I{}, std::integral_constant<int, 4>{})) return true;
    if (cfg == 16 && b1(I{}, std::integral_constant<int, 6>{})) return true;
  }
  auto go = [&](auto bt) -> bool {
    constexpr int BB = decltype(bt)::value;
    size_t lds = lb_lds_bytes<BB, 3>(a, pl);
    if (lds <= LDS_MAX) {
      if (!dry) hipLaunchKernelGGL((gemv_lds16<BB, 3>), dim3(G), dim3(LG_THREADS), lds, st, a, pl);
      return true;
    }
    lds = lb_lds_bytes<BB, 2>(a, pl);
    if (lds > LDS_MAX) return false;
    if (!dry) hipLaunchKernelGGL((gemv_lds16<BB, 2>), dim3(G), dim3(LG_THREADS), lds, st, a, pl);
    return true;
  };
  switch (a.B) {
    case 1: return go(std::integral_constant<int, 1>{});
    case 2: return go(std::integral_constant<int, 2>{});
    case 3: return go(std::integral_constant<int, 3>{});
    default: return go(std::integral_constant<int, 4>{});
  }
}
