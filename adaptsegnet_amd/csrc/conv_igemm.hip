// Implicit-GEMM convolution for gfx950 (MI355X): the fp32-input MFMA kernels
// (v_mfma_f32_32x32x2_f32, conv math F32) and the host side of every conv family (F32X3 on the
// bf16 MFMA, conv_x3.hpp / conv_x3r.hpp, the library default; bf16, conv_bf16*.hpp).
//
// One kernel template serves the three convolution products of the AdaptSegNet step
// (reference: every nn.Conv2d of model/deeplab_multi.py and model/discriminator.py):
//
//   FWD    C[m=(n,oh,ow)][co]       = sum_{k=(tap,ci)}  X[n, oh*s+dy(tap), ow*s+dx(tap), ci] * W[co][tap][ci]
//   DGRAD  C[m=(n,ih,iw)][ci]       = sum_{k=(tap,co)}  dY[n, (ih-dy)/s, (iw-dx)/s, co]       * W[co][tap][ci]
//   WGRAD  C[co][(tap,ci)]          = sum_{k=(n,oh,ow)} dY[n,oh,ow,co] * X[n, oh*s+dy, ow*s+dx, ci]
//
// A "tap" is one (kh, kw) position of one segment; (dy, dx) = (kh*dil - pad, kw*dil - pad).
// ASPP (Classifier_Module, model/deeplab_multi.py:106-121) is nseg = 4 segments whose
// taps are concatenated along K, so the four dilated 3x3 branches and their sum are a
// single GEMM.  Activations are NHWC; weights [Cout][KH][KW][Cin] per segment.
//
// Tiling: 256 threads (4 wave64s), block tile BM x BN, K step 16, two LDS stages with
// register staging (global loads of step k+1 are in flight while step k runs on the
// MFMA pipe).  LDS holds both operands k-major ([16][BM+pad]); each lane feeds the
// 32x32x2 MFMA with one ds_read_b32 per operand, which is conflict-free.  Small GEMM
// grids are split along K into fp32 slabs that a deterministic reduce kernel sums.
#include <atomic>
#include "conv_kernels.hpp"
#include "conv_thin.hpp"
#include <cstdlib>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace adaptseg {

// Split-K reduction + epilogue.  One thread per output element, slabs summed in order.
__global__ void splitk_reduce_kernel(const ConvParams p, const float *slab, int mode) {
  const size_t total = (size_t)p.M * p.N;
  for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < total;
       idx += (size_t)gridDim.x * blockDim.x) {
    float v = 0.f;
    for (int s = 0; s < p.splits; ++s) v += slab[(size_t)s * total + idx];
    int row = (int)(idx / p.N);
    int col = (int)(idx - (size_t)row * p.N);
    if (mode == MODE_WGRAD) {
      int seg = (int)fdiv((uint32_t)col, p.fd_nseg_k);
      int cc = col - seg * p.kseg;
      float *dst = seg == 0 ? p.dw[0] : seg == 1 ? p.dw[1] : seg == 2 ? p.dw[2] : p.dw[3];
      float *o = dst + (size_t)row * p.kseg + cc;
      *o = (p.flags & ADAPTSEG_EPI_ACCUMULATE) ? *o + v : v;
    } else {
      if (mode == MODE_FWD) {
        for (int s = 0; s < p.nseg; ++s) {
          const float *bp = s == 0 ? p.bias[0] : s == 1 ? p.bias[1] : s == 2 ? p.bias[2] : p.bias[3];
          if (bp) v += bp[col];
        }
      }
      if (p.flags & ADAPTSEG_EPI_ACCUMULATE) v += epi_prev(p, idx);
      if (p.flags & ADAPTSEG_EPI_RESIDUAL) v += epi_res(p, idx);
      v = epi_act(v, p.flags);
      if (p.flags & kEpiActGrad) v = epi_act_grad(v, p.aux[idx], p.flags);
      if (p.out) p.out[idx] = v;   // NULL: bf16 storage, only the copy below
      if (p.outb) epi_outb(p, (size_t)row, col, v);
    }
  }
}


__device__ __forceinline__ float4 bf4_of(uint2 u) {
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                     __uint_as_float(u.y & 0xffff0000u));
}

// Vectorised split-K reduction: 4 consecutive columns per thread (N % 4 == 0 and, for weight
// gradients, segments of kseg % 4 == 0), 32-bit indexing.  G split-groups per block: thread
// (g, lane) sums slabs g, g+G, ... of float4 `lane`, then the G partials are added in fixed
// order through LDS — deterministic, and a 256-split reduce is 16 loads deep, not 256.  The
// read-back operands (accumulate target, residual and its bitmap) are loaded raw BEFORE the slab
// loads, so their latency overlaps the slabs' instead of following it (round 4; bf16 images as
// raw words, converted at the use).
template <int G>
__global__ void __launch_bounds__(256) splitk_reduce4_kernel(const ConvParams p, const float *__restrict__ slab,
                                                             int mode, FastDiv fdn4) {
  constexpr int L = 256 / G;
  const uint32_t n4 = (uint32_t)p.N / 4;
  const uint32_t total4 = (uint32_t)p.M * n4;
  const float4 *s4 = reinterpret_cast<const float4 *>(slab);
  const int lane = threadIdx.x % L, g = threadIdx.x / L;
  const int flags = p.flags;
  const bool acc_f = flags & ADAPTSEG_EPI_ACCUMULATE;
  const bool res_f = mode != MODE_WGRAD && (flags & ADAPTSEG_EPI_RESIDUAL);
  __shared__ float4 red[G > 1 ? 256 : 1];
  for (uint32_t base = blockIdx.x * L; base < total4; base += gridDim.x * L) {  // block-uniform trip count
    const uint32_t i = base + lane;
    const bool fin = i < total4 && (G == 1 || g == 0);   // this thread finishes float4 i
    const uint32_t row = fin ? fdiv(i, fdn4) : 0;
    const int col = fin ? (int)(i - row * n4) * 4 : 0;
    float *o = nullptr;
    size_t idx = 0;
    float4 prev = make_float4(0.f, 0.f, 0.f, 0.f), resv = prev;
    uint2 prevb = make_uint2(0, 0), resb = prevb;
    uint32_t rw = ~0u;
    if (fin) {
      if (mode == MODE_WGRAD) {
        const int seg = (int)fdiv((uint32_t)col, p.fd_nseg_k);
        float *dst = seg == 0 ? p.dw[0] : seg == 1 ? p.dw[1] : seg == 2 ? p.dw[2] : p.dw[3];
        o = dst + (size_t)row * p.kseg + (col - seg * p.kseg);
        if (acc_f) prev = *reinterpret_cast<const float4 *>(o);
      } else {
        idx = (size_t)row * p.N + col;
        o = p.out ? p.out + idx : nullptr;   // NULL: bf16 storage, the output is p.outb
        if (acc_f) {
          if (o) prev = *reinterpret_cast<const float4 *>(o);
          else prevb = *reinterpret_cast<const uint2 *>(p.outb + idx);
        }
        if (res_f) {
          if (p.resb) resb = *reinterpret_cast<const uint2 *>(p.resb + idx);
          else resv = *reinterpret_cast<const float4 *>(p.res + idx);
          if (p.resbits) rw = p.resbits[idx >> 5] >> (idx & 31);   // 4 consecutive channels: 4 bits
        }
      }
    }
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (i < total4) {
#pragma unroll 8
      for (int s = g; s < p.splits; s += G) {
        const float4 t = s4[(size_t)s * total4 + i];
        v.x += t.x; v.y += t.y; v.z += t.z; v.w += t.w;
      }
    }
    if constexpr (G > 1) {
      red[threadIdx.x] = v;
      __syncthreads();
      if (g == 0)
        for (int q = 1; q < G; ++q) {
          const float4 t = red[q * L + lane];
          v.x += t.x; v.y += t.y; v.z += t.z; v.w += t.w;
        }
      __syncthreads();
    }
    if (!fin) continue;
    if (mode == MODE_WGRAD) {
      if (acc_f) {
        v.x += prev.x; v.y += prev.y; v.z += prev.z; v.w += prev.w;
      }
    } else {
      if (mode == MODE_FWD) {
        for (int s = 0; s < p.nseg; ++s) {
          const float *bp = s == 0 ? p.bias[0] : s == 1 ? p.bias[1] : s == 2 ? p.bias[2] : p.bias[3];
          if (bp) {
            const float4 b = *reinterpret_cast<const float4 *>(bp + col);
            v.x += b.x; v.y += b.y; v.z += b.z; v.w += b.w;
          }
        }
      }
      if (acc_f) {
        const float4 a = o ? prev : bf4_of(prevb);
        v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
      }
      if (res_f) {
        float4 a = p.resb ? bf4_of(resb) : resv;
        a.x = (rw & 1u) ? a.x : 0.f; a.y = (rw & 2u) ? a.y : 0.f; a.z = (rw & 4u) ? a.z : 0.f; a.w = (rw & 8u) ? a.w : 0.f;
        v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
      }
      v.x = epi_act(v.x, flags); v.y = epi_act(v.y, flags);
      v.z = epi_act(v.z, flags); v.w = epi_act(v.w, flags);
      if (flags & kEpiActGrad) {
        const float4 a = *reinterpret_cast<const float4 *>(p.aux + idx);
        v.x = epi_act_grad(v.x, a.x, flags); v.y = epi_act_grad(v.y, a.y, flags);
        v.z = epi_act_grad(v.z, a.z, flags); v.w = epi_act_grad(v.w, a.w, flags);
      }
    }
    if (o) *reinterpret_cast<float4 *>(o) = v;   // (NULL: bf16 storage, only the copy below)
    if (mode != MODE_WGRAD && p.outb) {
      if (p.outb_terms) {   // the F32X3 term images [row][3][N]
        uint2 th, tm, tl;
        split3(v, th, tm, tl);
        uint2 *ob = reinterpret_cast<uint2 *>(p.outb + (size_t)row * 3 * p.N + col);
        ob[0] = th;
        ob[p.N / 4] = tm;
        ob[p.N / 2] = tl;
      } else {
        __bf16 *ob = p.outb + idx;
        ob[0] = (__bf16)v.x; ob[1] = (__bf16)v.y; ob[2] = (__bf16)v.z; ob[3] = (__bf16)v.w;
      }
    }
  }
}

static bool aligned16(const void *q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; }
template <typename T>
static bool segs_aligned(T *const *w, int nseg) {
  for (int s = 0; s < nseg; ++s)
    if (!aligned16(w[s])) return false;
  return true;
}

// Bias gradient: db[seg][co] (+)= sum_m dY[m][co].  Each block sums a contiguous run of rows
// of the NHWC gradient with flat coalesced reads: for cout <= 256 thread t owns column t % cout
// and rows t / cout + j * (256 / cout) (so Cout = 19 uses 247 lanes, not 19 of 64); wider
// rows loop over their columns.  Partials are [split][cout], reduced by one wave per channel.
__global__ void __launch_bounds__(256) bias_grad_partial_kernel(const float *__restrict__ dy, int rows, int cout,
                                                                int rows_per_split, float *partial) {
  const int r0 = blockIdx.x * rows_per_split;
  const int r1 = min(rows, r0 + rows_per_split);
  __shared__ float red[256];
  if (cout <= 256) {
    const int rstep = 256 / cout;
    const int t = threadIdx.x;
    float s = 0.f;
    if (t < rstep * cout) {
      const float *src = dy + (size_t)r0 * cout + t;
      const int n = r1 - r0 - t / cout;  // rows left for this lane
#pragma unroll 8
      for (int j = 0; j < n; j += rstep) s += src[(size_t)j * cout];
    }
    red[t] = s;
    __syncthreads();
    if (t < cout) {
      float a = 0.f;
      for (int q = 0; q < rstep; ++q) a += red[t + q * cout];
      partial[(size_t)blockIdx.x * cout + t] = a;
    }
  } else {
    for (int col = threadIdx.x; col < cout; col += 256) {
      float s = 0.f;
#pragma unroll 8
      for (int r = r0; r < r1; ++r) s += dy[(size_t)r * cout + col];
      partial[(size_t)blockIdx.x * cout + col] = s;
    }
  }
}

// ~16K floats per block, at most 2048 blocks; rows per block a multiple of 256 / cout.
static void bias_grad_split(int rows, int cout, int *per, int *splits) {
  const int64_t want = ceil_div((int64_t)rows * cout, 16384);
  const int64_t s = std::max<int64_t>(1, std::min<int64_t>(want, 2048));
  const int rstep = cout <= 256 ? 256 / cout : 1;
  *per = (int)(ceil_div(ceil_div(rows, s), rstep) * rstep);
  *splits = (int)ceil_div(rows, *per);
}

// Four channels per lane (Cout % 4 == 0, 1024 % Cout == 0, 16-B aligned dY): 256 / (Cout / 4)
// row groups per block, each lane summing its column quad over every R-th row of the block's
// range in fp32, then the R group partials in fixed order through LDS — float4 loads instead of
// the kernel above's 4-B ones (DeeplabVGG's bias gradients: 6.8 ms per c4 step on it).
__global__ void __launch_bounds__(256) bias_grad_partial4_kernel(const float4 *__restrict__ dy, int rows, int c4,
                                                                 int rows_per_split, float4 *partial) {
  __shared__ float4 red[256];
  const int R = 256 / c4;                 // row groups
  const int t = threadIdx.x, cq = t % c4, g = t / c4;
  const int r0 = blockIdx.x * rows_per_split;
  const int r1 = min(rows, r0 + rows_per_split);
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (g < R) {
#pragma unroll 4
    for (int r = r0 + g; r < r1; r += R) {
      const float4 v = dy[(size_t)r * c4 + cq];
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
  }
  red[t] = a;
  __syncthreads();
  if (t < c4) {
    float4 sum = red[t];
    for (int q = 1; q < R; ++q) {
      const float4 v = red[t + q * c4];
      sum.x += v.x; sum.y += v.y; sum.z += v.z; sum.w += v.w;
    }
    partial[(size_t)blockIdx.x * c4 + t] = sum;
  }
}

static bool bias_grad_vec(const float *dy, int cout) {
  return cout % 4 == 0 && 1024 % cout == 0 && !(reinterpret_cast<uintptr_t>(dy) & 15);
}

struct BiasOut {
  float *db[4];
};

// One wave64 per channel: lanes stride over the splits (fp64), then a fixed shuffle tree.
__global__ void __launch_bounds__(256) bias_grad_final_kernel(const float *partial, int splits, int cout, BiasOut o,
                                                              int nseg, int accumulate) {
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (c >= cout) return;
  double s = 0.0;
  for (int i = lane; i < splits; i += 64) s += partial[(size_t)i * cout + c];
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  if (lane != 0) return;
  for (int g = 0; g < nseg; ++g) {
    float *d = o.db[g];
    if (!d) continue;
    d[c] = accumulate ? d[c] + (float)s : (float)s;
  }
}

// ------------------------------------------------------------------------------------
// Live timing (benchmark roofline): hipEvent pairs around selected launches.
// ------------------------------------------------------------------------------------
struct TimingState {
  std::mutex mu;
  bool enabled = false;
  bool mem_enabled = false;  // HBM-bound kernels (ids >= kTimingMemBase), adaptseg_timing_enable_mem
  bool stream_too = false;   // conv GEMMs: also bracket the stream time (adaptseg_timing_enable_stream)
  int selector = -1;
  // per slot: the measured pair (conv GEMMs: the kernel's execution, via hipExtLaunchKernel;
  // other kernels: stream events around the launch) and, for conv GEMMs under stream_too, a
  // stream-time pair recorded around the launch
  std::vector<std::pair<hipEvent_t, hipEvent_t>> events, sevents;
  std::vector<double> flops;  // algorithmic FLOPs (conv) or bytes (HBM-bound kernels) per launch
  std::vector<int> ids;
  std::vector<char> has_stream;
  size_t used = 0;
};
static TimingState g_timing;
// the execution-timed slot waiting for this thread's next launch_k (timing_begin_exec)
static thread_local int t_exec_slot = -1;

// Process-wide conv math (adaptseg_conv_set_math), default F32X3 (fp32-accurate on the bf16
// MFMA, conv_x3.hpp); F32 = the fp32-input MFMA kernels, BF16 = bf16 operands (config c5).
// Global, not thread-local: autograd runs backward on its own worker thread.
static std::atomic<int> g_conv_math{ADAPTSEG_MATH_F32X3};
int conv_math() { return g_conv_math.load(std::memory_order_relaxed); }

// Kernel-selection options (adaptseg_conv_set_option), initial values from the environment:
//   ADAPTSEG_OPT_X3H (ADAPTSEG_X3H): bits 1 / 2 / 4 put the F32X3 forward / data-gradient /
//     weight-gradient products the x3r tiles cover on igemm_x3h_kernel / igemm_x3hw_kernel
//     (conv_x3r.hpp) instead of the register-staged 128x128x16 kernel;
//   ADAPTSEG_OPT_G16_WIDE (ADAPTSEG_G16_WIDE): bit 1 = bf16 forward / data-gradient products with
//     N >= 256 and K >= 2048 on the 256x256x64 two-stage LDS-DMA tile, bit 2 = weight gradients
//     with Cout and N >= 256 on the 256x256 / 64-pixel tile (conv_bf16g.hpp).  Default 1: c5 +1.9 %
//     (profiles/r6/g16_wide_ab.txt); the weight-gradient tile measured -2.8 % on top of it.
#ifndef ADAPTSEG_X3H_DEFAULT
#define ADAPTSEG_X3H_DEFAULT 3
#endif
#ifndef ADAPTSEG_G16_WIDE_DEFAULT
#define ADAPTSEG_G16_WIDE_DEFAULT 1
#endif
static int env_int(const char *name, int dflt) {
  const char *e = std::getenv(name);
  return e && *e ? std::atoi(e) : dflt;
}
static std::atomic<int> g_opt_x3h{env_int("ADAPTSEG_X3H", ADAPTSEG_X3H_DEFAULT)};
static std::atomic<int> g_opt_g16_wide{env_int("ADAPTSEG_G16_WIDE", ADAPTSEG_G16_WIDE_DEFAULT)};
int x3h_mode() { return g_opt_x3h.load(std::memory_order_relaxed); }
int g16_wide_mode() { return g_opt_g16_wide.load(std::memory_order_relaxed); }

// one more slot (two event pairs), under g_timing.mu
static bool timing_grow() {
  hipEvent_t a, b, c, d;
  if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess || hipEventCreate(&c) != hipSuccess ||
      hipEventCreate(&d) != hipSuccess)
    return false;
  g_timing.events.push_back({a, b});
  g_timing.sevents.push_back({c, d});
  g_timing.flops.push_back(0.0);
  g_timing.ids.push_back(0);
  g_timing.has_stream.push_back(0);
  return true;
}

static int timing_slot(int kernel_id, double fl) {
  if (kernel_id >= kTimingMemBase) {
    if (!g_timing.mem_enabled) return -1;
  } else {
    if (!g_timing.enabled) return -1;
    if (g_timing.selector >= 0 && g_timing.selector != kernel_id) return -1;
  }
  std::lock_guard<std::mutex> lk(g_timing.mu);
  if (g_timing.used == g_timing.events.size() && !timing_grow()) return -1;
  const int slot = (int)g_timing.used++;
  g_timing.flops[slot] = fl;
  g_timing.ids[slot] = kernel_id;
  g_timing.has_stream[slot] = 0;
  return slot;
}

void timing_begin(int kernel_id, hipStream_t s, double fl, int *slot) {
  *slot = timing_slot(kernel_id, fl);
  if (*slot >= 0) (void)hipEventRecord(g_timing.events[*slot].first, s);
}

void timing_begin_exec(int kernel_id, hipStream_t s, double fl, int *slot) {
  *slot = timing_slot(kernel_id, fl);
  if (*slot < 0) return;
  t_exec_slot = *slot;
  if (g_timing.stream_too) {
    g_timing.has_stream[*slot] = 1;
    (void)hipEventRecord(g_timing.sevents[*slot].first, s);
  }
  *slot = -2 - *slot;   // timing_end: an execution-timed slot
}

bool timing_take_exec(hipEvent_t &start, hipEvent_t &stop) {
  if (t_exec_slot < 0) return false;
  start = g_timing.events[t_exec_slot].first;
  stop = g_timing.events[t_exec_slot].second;
  t_exec_slot = -1;
  return true;
}

void timing_end(int slot, hipStream_t s) {
  if (slot == -1) return;
  if (slot <= -2) {   // execution-timed: the launch recorded the pair
    const int i = -2 - slot;
    if (t_exec_slot == i) {   // no launch_k consumed it: nothing was timed
      t_exec_slot = -1;
      std::lock_guard<std::mutex> lk(g_timing.mu);
      g_timing.ids[i] = -1;
      return;
    }
    if (g_timing.has_stream[i]) (void)hipEventRecord(g_timing.sevents[i].second, s);
    return;
  }
  (void)hipEventRecord(g_timing.events[slot].second, s);
}

// ------------------------------------------------------------------------------------
// Host side
// ------------------------------------------------------------------------------------
static int validate(const adaptseg_conv_desc *d) {
  AS_CHECK_ARG(d, "null conv desc");
  AS_CHECK_ARG(d->n > 0 && d->c > 0 && d->h > 0 && d->w > 0 && d->k > 0, "conv: bad input/output dims");
  AS_CHECK_ARG(d->oh > 0 && d->ow > 0 && d->kh > 0 && d->kw > 0 && d->stride > 0, "conv: bad geometry");
  AS_CHECK_ARG(d->nseg >= 1 && d->nseg <= 4, "conv: nseg must be 1..4");
  AS_CHECK_ARG(d->nseg * d->kh * d->kw <= kMaxTaps, "conv: too many taps (%d)", d->nseg * d->kh * d->kw);
  for (int s = 0; s < d->nseg; ++s) {
    AS_CHECK_ARG(d->dil[s] >= 1 && d->pad[s] >= 0, "conv: bad pad/dil");
    int eh = (d->h + 2 * d->pad[s] - d->dil[s] * (d->kh - 1) - 1) / d->stride + 1;
    int ew = (d->w + 2 * d->pad[s] - d->dil[s] * (d->kw - 1) - 1) / d->stride + 1;
    AS_CHECK_ARG(eh == d->oh && ew == d->ow, "conv: output size %dx%d != expected %dx%d (seg %d)", d->oh,
                 d->ow, eh, ew, s);
  }
  int64_t in_elems = (int64_t)d->n * d->c * d->h * d->w;
  int64_t out_elems = (int64_t)d->n * d->k * d->oh * d->ow;
  AS_CHECK_ARG(in_elems < (1ll << 31) && out_elems < (1ll << 31), "conv: tensor too large for int32 indexing");
  return ADAPTSEG_OK;
}

static void fill_common(ConvParams &p, const adaptseg_conv_desc *d) {
  memset(&p, 0, sizeof(p));
  p.n = d->n; p.c = d->c; p.h = d->h; p.w = d->w;
  p.sxn = (int)d->in_stride[0]; p.sxc = (int)d->in_stride[1];
  p.sxh = (int)d->in_stride[2]; p.sxw = (int)d->in_stride[3];
  p.k = d->k; p.oh = d->oh; p.ow = d->ow;
  p.stride = d->stride;
  p.taps_per_seg = d->kh * d->kw;
  p.nseg = d->nseg;
  p.ntaps = p.taps_per_seg * d->nseg;
  int t = 0;
  for (int s = 0; s < d->nseg; ++s)
    for (int i = 0; i < d->kh; ++i)
      for (int j = 0; j < d->kw; ++j, ++t) {
        p.tap_dy[t] = (short)(i * d->dil[s] - d->pad[s]);
        p.tap_dx[t] = (short)(j * d->dil[s] - d->pad[s]);
      }
  p.kw_ = d->kw;
  p.kh_ = d->kh;
  for (int s = 0; s < 4; ++s) {
    p.pad_[s] = s < d->nseg ? d->pad[s] : 0;
    p.dil_[s] = s < d->nseg ? d->dil[s] : 1;
  }
  p.fd_taps = make_fastdiv(p.taps_per_seg);
  p.fd_kw = make_fastdiv(d->kw);
  p.fd_c = make_fastdiv(d->c);
  p.fd_k = make_fastdiv(d->k);
  p.fd_ow = make_fastdiv(d->ow);
  p.fd_oh = make_fastdiv(d->oh);
  p.fd_w = make_fastdiv(d->w);
  p.fd_hw = make_fastdiv(d->h);
}

double conv_flops(const adaptseg_conv_desc *d) {
  return 2.0 * d->n * d->oh * d->ow * (double)d->k * d->c * d->kh * d->kw * d->nseg;
}

// Bytes of the split-K slabs [splits][M][N] fp32, 256-B aligned (the tile counters follow).
size_t splitk_slab_bytes(const Plan &pl) {
  return ((size_t)pl.p.splits * pl.p.M * pl.p.N * sizeof(float) + 255) / 256 * 256;
}

// Row tile of the plan's kernel (the fused BN statistics count one partial per row tile).
int plan_bm(const Plan &pl) {
  if (pl.g16) return pl.g16_bm;
  if (pl.x3r) return pl.mode == MODE_WGRAD ? pl.x3r_bm : 256;
  if (pl.x3h) return pl.mode == MODE_WGRAD ? pl.x3r_bm : 256;
  return (pl.bf16 || pl.x3) ? 128 : kCfgBM[pl.cfg];
}

// F32X3 maths with the caller's term images of the activation operand(s) (the _x forms'
// copies: the three bf16 terms, pixel-interleaved [n][h][w][3][c]): the product moves to the x3r
// kernel, which reads them by LDS-DMA instead of splitting fp32 rows in-kernel (F32X3_PRESPLIT:
// it is there already; it then skips its per-call copy).  Re-plans the grid.
static void x3_terms_flags(Plan &pl) {
  pl.x3g = pl.x3r = pl.x3ext = true;
  pl.x3h = false;
  if (pl.mode == MODE_WGRAD) pl.x3r_bm = pl.p.M >= 256 ? 256 : 128;   // (make_plan's choice; x3h set 128)
  // weight gradients under the default maths run on the side stream beside the main chain's
  // register-staged blocks: the 128-row tile (96 KB LDS, <= 128 VGPRs) leaves a CU room for one
  // of them, the 256-row one (144 KB) does not — except for Cout >= 1024 (DeeplabVGG's fc6 / fc7,
  // whose main chain runs on the term-image kernel too): there the 256-row tile halves the dY
  // re-reads, c4 +0.4 % over three alternating pairs (profiles/r5/x3r_wgrad_bm256_ab.txt)
#ifndef ADAPTSEG_X3R_WGRAD_BM256_MIN_COUT
#define ADAPTSEG_X3R_WGRAD_BM256_MIN_COUT 1024   // 0: always the 128-row tile under F32X3
#endif
  if (pl.mode == MODE_WGRAD && conv_math() == ADAPTSEG_MATH_F32X3 &&
      !(ADAPTSEG_X3R_WGRAD_BM256_MIN_COUT > 0 && pl.p.M >= ADAPTSEG_X3R_WGRAD_BM256_MIN_COUT))
    pl.x3r_bm = 128;
}
static void x3_terms(Plan &pl) {
  if (!copies_are_terms() || !pl.fast || !pl.x3 || !pl.x3r_ok || !pl.act_ext) return;
  if (pl.mode == MODE_WGRAD && !pl.act_ext2) return;
  x3_terms_flags(pl);
  set_splits(pl);
}

// Grid decomposition: tiles, then split K until the grid has ~2 blocks per CU while keeping
// >= 8 K-steps per split.  Depends on the K step of the chosen kernel (pl.bk).
void set_splits(Plan &pl) {
  ConvParams &p = pl.p;
  if (!pl.fast) pl.s2 = pl.bf16 = pl.x3 = pl.x3g = pl.x3r = pl.x3h = pl.g16 = false;
  if (!pl.fast && pl.cfg == 8) pl.cfg = 0;  // cfg 8 is built for vector FAST operands only
  const int bm = plan_bm(pl);
  const int bn = pl.g16 ? pl.g16_bn : pl.bf16 ? pl.bf16_bn : pl.x3 ? x3_bn(pl.mode) : kCfgBN[pl.cfg];
  pl.bk = pl.g16 ? pl.g16_bk : pl.bf16 ? 64 : (pl.x3r || pl.x3h) ? kX3rBK : pl.x3 ? kX3BK : pl.fast ? fast_bk(pl.cfg) : BK;
  if (pl.s2) {  // rows of the largest parity class; K of the largest tap subset; no K split
    p.M = p.n * ((p.h + 1) / 2) * ((p.w + 1) / 2);
    p.K = ((p.kh_ + 1) / 2) * ((p.kw_ + 1) / 2) * p.k;
  } else if (pl.mode == MODE_DGRAD) {
    p.M = p.n * p.h * p.w;
    p.K = p.ntaps * p.k;
  }
  pl.tiles = (int)(ceil_div(p.M, bm) * ceil_div(p.N, bn));
  const int nkt = (int)ceil_div(p.K, pl.bk);
  // Split targets (measured on the step, not per shape; tools/ab.sh):
  //  * weight gradients: ~512 blocks (two per CU), rounded down — 384 / 768 / 1024 measured
  //    -3.2 / -2.3 / -2.5 % at c2 and -2.8 / -3.1 / -3.2 % at c3;
  //  * fwd / data-grad: only grids of at most one block per CU (<= 256 tiles) split, to ~512
  //    blocks — one resident block per CU hides no latency (c3 target-domain layer3: +0.6 %
  //    step); splitting grids of up to two blocks per CU measured 2 % slower, a threshold of
  //    129 tiles -0.1 % c2 / -1.2 % c3.
  // >= 4 K-steps per split keeps the slab traffic small next to the GEMM.
  // Rounding: the blocks of a split grid are equal work, so the grid takes (the most blocks any
  // CU runs) x (one block's K range); tiles * splits must not overshoot a multiple of the CU
  // count: ceil(512 / 36) = 15 splits puts 3 blocks on 28 CUs (0.2 units) where 14 puts at most
  // 2 on every CU (0.143) — round down.
  constexpr int kSplitTarget = 512;
  // F32X3 weight gradients (side stream) split to ~384 blocks (1.5 per CU), not 512: a full
  // 2-per-CU grid of 16-wave blocks holds every CU for a whole split, and the main stream's
  // short BN / split-K kernels then wait for CU slots.  384 measured c2 +2.4 %, c3 +2.6 %
  // (256 / 320 / 448 / 1024: +1.2 / +1.7 / +2.0 / +0.1 % at c2).  Rounding the split count to
  // nearest instead of down measured -0.2..-0.8 % (profiles/r3/x3_wgrad_split_rounding_ab.txt).
#ifndef ADAPTSEG_X3_WGRAD_TARGET
#define ADAPTSEG_X3_WGRAD_TARGET 384   // (a compile-time knob of experiment builds, EXTRA=-D...)
#endif
  // (the environment variable ADAPTSEG_X3_WGRAD_TARGET overrides it, for A/B runs)
  static const int kX3WgradTarget = env_int("ADAPTSEG_X3_WGRAD_TARGET", ADAPTSEG_X3_WGRAD_TARGET);
  // The LDS-DMA bf16 weight gradient (side stream) to ~256 blocks: half the split-K slab
  // traffic of 512, c5 +1.8 % same box (37.30 / 37.30 / 37.29 vs 36.64 / 36.65 / 36.62,
  // tools/dbg/ab_lib.sh).
  constexpr int kG16WgradTarget = 256;
  // (the term-image F32X3 weight gradient picks its own split count below)
  const int target = (pl.mode == MODE_WGRAD && pl.g16) ? kG16WgradTarget
                     : (pl.mode == MODE_WGRAD && pl.x3)            ? kX3WgradTarget
                                                                   : kSplitTarget;
  // the LDS-DMA bf16 / x3r kernels run one block per CU: split only grids under half the CUs
  // (the 256x256 bf16 tile, one block per CU: split under 256 tiles, like x3r)
  const bool g16w = pl.g16 && pl.g16_bm == 256 && pl.g16_bn == 256;
  const int split_below = pl.mode == MODE_WGRAD ? target : (pl.x3r || pl.x3h || g16w) ? 256 : pl.g16 ? 128 : 257;
  int splits = 1;
  if (pl.mode == MODE_WGRAD && (pl.x3r || pl.x3h)) {
    // one 8-wave block per CU: the grid takes ceil(tiles * s / 256) rounds of 1/s of the K range,
    // so pick the split count s (<= 256, >= 32 K steps each) with the fewest such units — e.g.
    // layer4.conv2 (144 tiles of 128 rows): s = 1 leaves 112 CUs idle for the whole launch
    // (MFMA busy 0.315 in isolation), s = 7 runs 4 rounds of 1/7 (0.57 of the s = 1 time).
    // (Round 4 capped s at 16: the 1x1 weight gradients, 1-8 tiles over K = 32-131k pixels, then
    // ran 16-128 blocks on 256 CUs — layer1 at 4-33 TF/s, layer3's 1x1 at 107-112.)
#ifndef ADAPTSEG_X3R_WGRAD_MIN_KSTEPS
#define ADAPTSEG_X3R_WGRAD_MIN_KSTEPS 32
#endif
    double best = 1e30;
    for (int s = 1; s <= 256 && (s == 1 || nkt / s >= ADAPTSEG_X3R_WGRAD_MIN_KSTEPS); ++s) {
      const double t = (double)ceil_div((int64_t)pl.tiles * s, 256) / s;
      if (t < best * 0.97) {
        best = t;
        splits = s;
      }
    }
  } else if (pl.tiles < split_below && !pl.s2) {
    splits = std::max(1, ((pl.g16 || pl.x3r || pl.x3h) && pl.mode != MODE_WGRAD ? 256 : target) / pl.tiles);
    splits = std::min(splits, std::max(1, nkt / 4));
    splits = std::min(splits, 256);
  }
  int per = (int)ceil_div(nkt, splits);
  splits = (int)ceil_div(nkt, per);
  p.splits = splits;
  p.ktiles_per_split = per;
  pl.slab_bytes = splits > 1 ? splitk_slab_bytes(pl) : 0;
  if (pl.bf16) pl.slab_bytes += bf16_pre_bytes(pl);
  if (pl.x3) pl.slab_bytes += x3_pre_bytes(pl);
}

int make_plan(const adaptseg_conv_desc *d, int op, Plan &pl) {
  int st = validate(d);
  if (st) return st;
  ConvParams &p = pl.p;
  fill_common(p, d);
  pl.mode = op;
  pl.act_ext = pl.act_ext2 = nullptr;
  pl.wpack_ext = nullptr;
  const bool nhwc_in = d->in_stride[1] == 1;
  if (op == ADAPTSEG_CONV_FWD) {
    p.M = d->n * d->oh * d->ow;
    p.N = d->k;
    p.K = p.ntaps * d->c;
    p.kseg = p.taps_per_seg * d->c;
    pl.va = nhwc_in && d->c % 4 == 0;
    pl.vb = d->c % 4 == 0;
    pl.cfg = p.N <= 32 ? 1 : (p.N <= 64 ? 4 : 0);
  } else if (op == ADAPTSEG_CONV_BWD_DATA) {
    p.M = d->n * d->h * d->w;
    p.N = d->c;
    p.K = p.ntaps * d->k;
    p.kseg = p.taps_per_seg * d->c;
    pl.va = d->k % 4 == 0;
    pl.vb = d->c % 4 == 0;
    pl.cfg = p.N <= 32 ? 1 : (p.N <= 64 ? 4 : 0);
  } else if (op == ADAPTSEG_CONV_BWD_WEIGHT) {
    p.M = d->k;
    p.N = p.ntaps * d->c;
    p.K = d->n * d->oh * d->ow;
    p.kseg = p.taps_per_seg * d->c;
    pl.va = d->k % 4 == 0;
    pl.vb = nhwc_in && d->c % 4 == 0;
    // M' = Cout rows, N' = taps*Cin columns: pick the tile that wastes the least MFMA work
    pl.cfg = p.M <= 32 ? 2 : p.M <= 64 ? (p.N <= 64 ? 5 : 3) : (p.N <= 64 ? 4 : 0);
  } else {
    set_error("conv: bad op %d", op);
    return ADAPTSEG_ERR_ARG;
  }
  // 128x128 tile at BK 16 (cfg 6: half the LDS, shorter K steps) measured faster than BK 32
  // for multi-tap weight gradients (+2-8 %, per-shape conv bench, profiles/r1/conv_cfg_ab.txt).
  if (pl.cfg == 0 && op == ADAPTSEG_CONV_BWD_WEIGHT && d->kh * d->kw > 1) pl.cfg = 6;
  // Forward products on the occupancy-3 BK-16 tile (cfg 8): +0.9 % c2 / +0.8 % c3 end to end
  // (two alternating runs each) and 0.67 -> 0.69 of peak on the dominant forward symbol.  The
  // weight gradients stay on cfg 6 (cfg 8 there: -0.7 %).  Non-FAST / per-element / stride-2
  // plans fall back to cfg 0 below.  Measured and rejected: data gradient on cfg 6 (BK16, 4
  // blocks/CU instead of 2) -1.1 % c2 / -0.7 % c3; 1x1 weight gradients on cfg 6 -0.3 % /
  // -1.1 %, on cfg 8 -1.2 % / -1.8 %.
  // Stride-1 1x1 vector data gradients on the occupancy-3 BK-16 tile too (cfg 8: 121 VGPRs,
  // no AGPRs; the cfg-0 build needs 2 waves per SIMD): +2.5 % c2 / +1.8 % c3 / +-0 c5.  Every
  // stride-1 product (3x3 too) on it measured +1.6 % c2 but -4.4 % c3, so the 3x3 ones stay on
  // cfg 0 (its min-blocks-2 build, conv_launch_body.inc).
  if (pl.cfg == 0 && op == ADAPTSEG_CONV_BWD_DATA && d->stride == 1 && d->k % 16 == 0 && d->c % 4 == 0 &&
      d->kh * d->kw == 1)
    pl.cfg = 8;
  if (pl.cfg == 0 && op == ADAPTSEG_CONV_FWD) pl.cfg = 8;
  p.fd_nseg_k = make_fastdiv(p.kseg);
  pl.flops = conv_flops(d);
  // FAST path eligibility (alignment re-checked at launch).  Vector operands need tile-
  // uniform taps and float4 rows; otherwise the per-element (AE / BE) variants apply.
  const int fbk = fast_bk(pl.cfg);
  pl.s2 = pl.ae = pl.be = false;
  if (op == ADAPTSEG_CONV_FWD) {
    if (nhwc_in && d->c % fbk == 0) {
      pl.fast = true;
    } else {
      pl.fast = d->nseg == 1;
      pl.ae = true;
      pl.be = p.kseg % 4 != 0 || p.K % fbk != 0;  // vector W rows need no K tail
    }
  } else if (op == ADAPTSEG_CONV_BWD_DATA) {
    const bool s2 = d->stride == 2 && d->nseg == 1 && d->dil[0] == 1;
    pl.ae = d->k % fbk != 0;
    pl.be = d->c % 4 != 0;
    pl.fast = d->stride == 1 || (s2 && !pl.ae);
    pl.s2 = s2 && pl.fast;
  } else {
    pl.fast = true;
    pl.ae = d->k % 4 != 0;
    pl.be = !(nhwc_in && d->c % 4 == 0);
  }
  // bf16 conv math: the vector FAST cases whose K tiles of 64 stay inside one tap
  pl.bf16 = pl.g16 = false;
  const bool bf16_math = conv_math() == ADAPTSEG_MATH_BF16 || conv_math() == ADAPTSEG_MATH_BF16_WIDE;
  if (bf16_math && pl.fast && !pl.ae && !pl.be) {
    if (op == ADAPTSEG_CONV_FWD) pl.bf16 = d->c % 64 == 0;
    else if (op == ADAPTSEG_CONV_BWD_DATA) pl.bf16 = d->k % 64 == 0;
    else pl.bf16 = true;
  }
  // F32X3 conv math: the vector FAST cases whose 16-deep K tiles stay inside one tap
  pl.x3 = pl.x3g = pl.x3r = pl.x3r_ok = pl.x3ext = pl.x3h = false;
  pl.x3r_bm = 256;
  const bool x3_math = conv_math() == ADAPTSEG_MATH_F32X3 || conv_math() == ADAPTSEG_MATH_F32X3_PRESPLIT;
  if (x3_math && pl.fast && !pl.ae && !pl.be) {
    if (op == ADAPTSEG_CONV_FWD) pl.x3 = d->c % kX3BK == 0;
    else if (op == ADAPTSEG_CONV_BWD_DATA) pl.x3 = d->k % kX3BK == 0;
    else pl.x3 = true;
    // 256x128 tiles with 32-deep steps on pre-split term images (conv_x3r.hpp): a 32-deep
    // step inside one tap; weight gradients in 16-B channel chunks of both operands
    if (pl.x3) {
      if (op == ADAPTSEG_CONV_FWD) pl.x3r_ok = d->c % kX3rBK == 0;
      else if (op == ADAPTSEG_CONV_BWD_DATA) pl.x3r_ok = d->k % kX3rBK == 0;
      else pl.x3r_ok = d->c % 8 == 0 && d->k % 8 == 0;
      if (op == ADAPTSEG_CONV_BWD_WEIGHT) pl.x3r_bm = d->k >= 256 ? 256 : 128;
    }
    // F32X3_PRESPLIT: every such product on the term-image kernel, the images made per call
    // unless the caller supplies them; F32X3 (default): on it only when the caller does (x3_terms:
    // the engine's layer 3-4 conv2 products, whose term images the BN passes write).  Per-call
    // images under F32X3 measured slower for the multi-tap weight gradients (c2 -1.4 %,
    // profiles/r3/x3r_wgrad_taps_ab.txt); experiments/r3_rejected.patch keeps that build.
    if (pl.x3 && conv_math() == ADAPTSEG_MATH_F32X3_PRESPLIT) pl.x3g = pl.x3r = pl.x3r_ok;
    // F32X3: products on the x3r tiles with the fp32 operands split in-kernel (igemm_x3h_kernel,
    // igemm_x3hw_kernel), by ADAPTSEG_X3H bit 1 (forward) / 2 (data gradient) / 4 (weight gradient)
    // Forward / data gradient only at K >= 512 (256 until late round 6; per shape, tools/conv_bench.py: the layer-1 1x1
    // products with K = 64 / 128 run slower on the 256-row tile — two to four K steps against its
    // prologue and epilogue) and not on the stride-2 parity classes (D.conv2's data gradient 449 ->
    // 523 us); the larger products gain 4-12 % (l4.ds forward 854 -> 775 us).
    // (round-6 final program: 512 — the K 256 products back on the staged kernel averaged +0.4 %
    // over 256 on two boxes, profiles/r6/x3h_min_k_ab.txt; ADAPTSEG_X3H_MIN_K for A/B runs)
    static const int x3h_min_k = env_int("ADAPTSEG_X3H_MIN_K", 512);
    const bool x3h_fd = p.K >= x3h_min_k && !(op == ADAPTSEG_CONV_BWD_DATA && d->stride == 2);
    if (pl.x3 && pl.x3r_ok && conv_math() == ADAPTSEG_MATH_F32X3 &&
        ((op == ADAPTSEG_CONV_FWD && (x3h_mode() & 1) && x3h_fd) ||
         (op == ADAPTSEG_CONV_BWD_DATA && (x3h_mode() & 2) && x3h_fd) ||
         (op == ADAPTSEG_CONV_BWD_WEIGHT && (x3h_mode() & 4)))) {
      pl.x3h = true;
      if (op == ADAPTSEG_CONV_BWD_WEIGHT) pl.x3r_bm = 128;   // igemm_x3hw_kernel<128> (conv_launch_x3.hip)
    }
  }
  if (pl.x3) pl.cfg = 0;
  if (pl.bf16) {
    pl.cfg = 0;
    // 128x256 (8 waves) halves the refetch of the gathered A operand but measured no faster
    // (c5 27.6 vs 27.7 images/s, per-shape within +-5 %): only with ADAPTSEG_MATH_BF16_WIDE
    const bool w256 = conv_math() == ADAPTSEG_MATH_BF16_WIDE;
    pl.bf16_bn = (w256 && op != ADAPTSEG_CONV_BWD_WEIGHT && p.N >= 256) ? 256 : 128;
    // forward / data gradients with N >= 64 on the LDS-DMA kernel (conv_bf16g.hpp): 128x256 tiles
    // when N >= 256 (the activation operand is fetched once per tap), else 256x128 — at N = 64
    // (layer1, D.conv2's stride-2 data gradient) with half the column tile idle, still faster than
    // the register-staged bf16 kernel: l1.conv2 48 -> 40 us, D.conv2 data gradient 204 -> 171,
    // c5 +0.8 % (profiles/r5/g16_min_n64_ab.txt; 128: the round-4 threshold)
#ifndef ADAPTSEG_G16_MIN_N
#define ADAPTSEG_G16_MIN_N 64
#endif
    if (op != ADAPTSEG_CONV_BWD_WEIGHT && p.N >= ADAPTSEG_G16_MIN_N) {   // stride-2 data gradients by parity class too
      pl.g16 = true;
      pl.g16_bm = p.N >= 256 ? 128 : 256;
      pl.g16_bn = p.N >= 256 ? 256 : 128;
      // K step: 64 (one block per CU) for K >= 2048, else 32 (two blocks per CU: one block's
      // prologue / epilogue overlaps the other's loop on short-K products) — per shape
      // (tools/conv_bench.py, kernel time): l3.conv2 (K 2304) 706 vs 675 TF/s, l4.conv3 forward
      // (K 512) 483 vs 625, l4.conv1 data gradient (K 512) 488 vs 631
      pl.g16_bk = (p.K >= 2048 && !pl.s2) ? 64 : 32;   // parity classes: short K, step 32
      // 256x256x64, two stages (ADAPTSEG_G16_WIDE_MIN_K: the smallest K, for A/B runs; 512 / 256
      // speed the 1x1 products up alone, -1.3 % conv time, but cost the c5 step 0.3 %:
      // profiles/r6/g16_wide_min_k_ab.txt)
      static const int wide_min_k = env_int("ADAPTSEG_G16_WIDE_MIN_K", 2048);
      // ... and only where its grid holds >= 128 tiles (grids of 128-255 tiles split K to ~256
      // blocks, set_splits): per shape l4.conv2 899 -> 1068 TF/s on it, l3.conv2 at c5's source
      // geometry (225 tiles) 691 -> 893, at the c2 geometry (128 tiles) unsplit 712 -> 551
      // (profiles/r6/g16_wide_ab.txt); the c5 step is within +-0.3 % of a 256-tile threshold
      static const int wide_min_tiles = env_int("ADAPTSEG_G16_WIDE_MIN_TILES", 128);   // (under 256: split-K to 256 blocks)
      const int64_t wide_tiles = ceil_div(p.M, 256) * ceil_div(p.N, 256);
      if ((g16_wide_mode() & 1) && p.N >= 256 && p.K >= wide_min_k && !pl.s2 && wide_tiles >= wide_min_tiles) {
        pl.g16_bm = 256;
        pl.g16_bk = 64;
      }
      // (256x256x32 tiles, one block per CU, measured slower: c5 -10 % / -2.4 % with the weight
      // gradients only, profiles/r3/bf16_wide_tiles_ab.txt; experiments/r3_rejected.patch)
    }
    // weight gradients with 16-B channel chunks (Cin % 8 == 0, Cout % 8 == 0) on the LDS-DMA
    // weight-gradient kernel: {128,256}x128 tiles, K steps of 32 output pixels
    // (its pixel walk keeps 32-bit element offsets: operands of < 2^31 elements, g16_wgrad_fits)
    const bool g16_wgrad_fits = ((int64_t)p.n * p.oh * p.ow + 64) * p.k < INT32_MAX &&
                                ((int64_t)p.n + 1) * p.h * p.w * p.c < INT32_MAX;
    if (op == ADAPTSEG_CONV_BWD_WEIGHT && d->c % 8 == 0 && d->k % 8 == 0 && g16_wgrad_fits) {
      pl.g16 = true;
      pl.g16_bm = d->k >= 256 ? 256 : 128;   // 256 rows: dY read once per column tile
      pl.g16_bn = 128;
      pl.g16_bk = 32;
      // 256x256 with 64-pixel K steps (16 waves, two stages: ADAPTSEG_OPT_G16_WIDE)
      if ((g16_wide_mode() & 2) && d->k >= 256 && p.N >= 256) {
        pl.g16_bn = 256;
        pl.g16_bk = 64;
      }
    }
  }
  // cfg 8 (occupancy-3 BK-16 tile) exists for vector FAST fwd / weight-grad products only
  if (pl.cfg == 8 && (!pl.fast || pl.ae || pl.be || pl.s2)) {
    if (op == ADAPTSEG_CONV_BWD_DATA) {  // screened above: unreachable unless misaligned
      set_error("conv: data-gradient plan on cfg 8 without vector FAST operands");
      return ADAPTSEG_ERR_ARG;
    }
    pl.cfg = 0;
  }
  set_splits(pl);
  return ADAPTSEG_OK;
}

int kernel_id(const Plan &pl, int mode) {
  // 88 / 89: the FAST cfg-8 stride-2 ids, which never occur (cfg 8 has no stride-2 form)
  if (pl.x3r) return 100 * mode + 88 + ((mode == MODE_WGRAD ? pl.x3r_bm == 128 : pl.s2) ? 1 : 0);
  // 86 / 87: the FAST cfg-8 per-element ids, which never occur (cfg 8 takes vector operands only)
  if (pl.x3h) return 100 * mode + 86 + ((mode == MODE_WGRAD ? pl.x3r_bm == 128 : pl.s2) ? 1 : 0);
  if (pl.g16 && mode == MODE_WGRAD) return 100 * mode + (pl.g16_bn == 256 ? 85 : pl.g16_bm == 256 ? 98 : 99);
  if (pl.g16 && pl.s2) return 100 * mode + (pl.g16_bn == 256 ? 92 : 93);
  // 85: the FAST cfg-8 id with per-element B, which never occurs (cfg 8: vector operands only)
  if (pl.g16 && pl.g16_bm == 256 && pl.g16_bn == 256) return 100 * mode + 85;
  if (pl.g16) return 100 * mode + (pl.g16_bk == 64 ? (pl.g16_bn == 256 ? 97 : 98) : (pl.g16_bn == 256 ? 94 : 99));
  if (pl.bf16) return 100 * mode + 90 + (pl.s2 ? 1 : 0) + (pl.bf16_bn == 256 ? 2 : 0);
  if (pl.x3) return 100 * mode + 95 + (pl.s2 ? 1 : 0);
  // FAST: 4 + (S2 ? 4 : 0) + (AE ? 2 : 0) + (BE ? 1 : 0)  ->  4..11 (S2 variants 8, 9)
  if (pl.fast) return 100 * mode + 10 * pl.cfg + 4 + (pl.s2 ? 4 : 0) + (pl.ae ? 2 : 0) + (pl.be ? 1 : 0);
  return 100 * mode + 10 * pl.cfg + (pl.va ? 2 : 0) + (pl.vb ? 1 : 0);
}

// Split-K outputs: the operands of the final sum are 16-byte aligned float4 rows for
// splitk_reduce4_kernel (else the scalar splitk_reduce_kernel).  Folding the sum into the
// last-arriving split (per-tile arrival counter) measured slower — c2 25.86 vs 26.66 images/s,
// c5 35.70 vs 38.56 (profiles/r3/splitk_fold_ab.txt): a 128x128 fp32 slab is 64 KB, so one
// reducer block reads splits x 64 KB serially at the tail of the launch, where the separate
// reduce spreads it over the chip (experiments/r3_rejected.patch keeps that build).

static bool splitk_vec(const ConvParams &q, const float *slab, const float *final_out, int mode) {
  bool vec = q.N % 4 == 0 && aligned16(slab);
  if (mode == MODE_WGRAD) {
    vec = vec && q.kseg % 4 == 0;
    for (int g = 0; g < q.nseg; ++g) vec = vec && aligned16(q.dw[g]);
  } else {
    vec = vec && aligned16(final_out) && aligned16(q.outb) &&
          (!(q.flags & ADAPTSEG_EPI_RESIDUAL) || aligned16(q.res ? (const void *)q.res : (const void *)q.resb)) &&
          (!(q.flags & kEpiActGrad) || aligned16(q.aux));
    if (mode == MODE_FWD)
      for (int g = 0; g < q.nseg; ++g) vec = vec && (!q.bias[g] || aligned16(q.bias[g]));
  }
  return vec;
}

// The split-K sum of one product (q.out: the final output; slab: its splits' partial outputs)
static int splitk_sum(const ConvParams &q, const float *slab, int mode, hipStream_t s) {
  const size_t total = (size_t)q.M * q.N;
  const bool vec = splitk_vec(q, slab, q.out, mode);
  int slot;  // the slabs + read-modify-write operands in, the output out
  const int extra = (q.flags & ADAPTSEG_EPI_ACCUMULATE ? 1 : 0) +
                    (mode != MODE_WGRAD && (q.flags & ADAPTSEG_EPI_RESIDUAL) ? 1 : 0) +
                    (mode != MODE_WGRAD && (q.flags & kEpiActGrad) ? 1 : 0);
  timing_begin(kTSplitkReduce, s, 4.0 * (double)total * (q.splits + 1 + extra), &slot);
  if (vec) {
    const FastDiv fdn4 = make_fastdiv((uint32_t)q.N / 4);
    const int G = q.splits >= 64 ? 16 : q.splits >= 16 ? 4 : 1;
    // grid cap: 512 / 1024 / 8192 measured within +-0.2 % (round 3); ADAPTSEG_SPLITK_MAX_BLOCKS
    // for A/B runs (the block-stride loop covers any cap)
    static const int max_blocks = env_int("ADAPTSEG_SPLITK_MAX_BLOCKS", 8192);
    const int blocks = (int)std::min<size_t>(ceil_div(total / 4, 256 / G), (size_t)std::max(1, max_blocks));
    if (G == 16) splitk_reduce4_kernel<16><<<blocks, 256, 0, s>>>(q, slab, mode, fdn4);
    else if (G == 4) splitk_reduce4_kernel<4><<<blocks, 256, 0, s>>>(q, slab, mode, fdn4);
    else splitk_reduce4_kernel<1><<<blocks, 256, 0, s>>>(q, slab, mode, fdn4);
  } else {
    int blocks = (int)std::min<size_t>(ceil_div(total, 256), 4096);
    splitk_reduce_kernel<<<blocks, 256, 0, s>>>(q, slab, mode);
  }
  timing_end(slot, s);
  AS_CHECK_LAUNCH("splitk_reduce");
  return ADAPTSEG_OK;
}

// Deferred split-K sums (adaptseg_splitk_flush): per stream, in launch order.  A weight
// gradient's sum only feeds the optimiser, so its launch can wait until the backward has
// queued every weight-gradient GEMM.  Removing the sums outright is worth c2 +8 %, c5 +3 %
// (profiles/r6/sol_diag.txt, about twice their kernel time); deferring them to the end of the
// backward measured c2 -1.0 %, c5 -1.3 % (profiles/r6/splitk_defer_ab.txt: the work stays on
// the weight-gradient stream, now at its tail), so the engine keeps it off (ADAPTSEG_DEFER_SPLITK).
struct PendingSum {
  ConvParams q;
  const float *slab;
  int mode;
};
static std::mutex g_pending_mu;
static std::unordered_map<hipStream_t, std::vector<PendingSum>> g_pending;

int run_plan(Plan &pl, int mode, void *ws, size_t ws_bytes, hipStream_t s, bool defer) {
  float *final_out = pl.p.out;
  if (!ws || ws_bytes < pl.slab_bytes) {
    if (pl.slab_bytes) {
      set_error("conv: workspace %zu < required %zu", ws_bytes, pl.slab_bytes);
      return ADAPTSEG_ERR_WORKSPACE;
    }
  }
  // workspace: [weight pack / operand copies (F32X3, bf16)][split-K slabs][tile counters]
  const size_t pre = pl.x3 ? x3_pre_bytes(pl) : pl.bf16 ? bf16_pre_bytes(pl) : 0;
  float *slab = nullptr;
  if (pl.p.splits > 1) {
    slab = reinterpret_cast<float *>(reinterpret_cast<char *>(ws) + pre);
    pl.p.out = slab;
  }
  hipError_t e;
  int slot;
  if (pl.bf16 || pl.x3) {
    // weight pack (+ operand copies) first, outside the timed bracket: the live roofline
    // times the GEMM kernel alone, as rocprof reports it
    e = pl.x3 ? prep_x3(pl, ws, s) : prep_bf16(pl, ws, s);
    if (e == hipSuccess) {
      timing_begin_exec(kernel_id(pl, mode), s, pl.flops, &slot);
      e = pl.x3 ? launch_x3(pl, ws, s) : launch_bf16(pl, ws, s);
      timing_end(slot, s);
    }
  } else {
    timing_begin_exec(kernel_id(pl, mode), s, pl.flops, &slot);
    if (mode == MODE_FWD) e = launch_fwd(pl, s);
    else if (mode == MODE_DGRAD) e = launch_dgrad(pl, s);
    else e = launch_wgrad(pl, s);
    timing_end(slot, s);
  }
  if (e != hipSuccess) {
    set_error("igemm launch: %s", hipGetErrorString(e));
    return ADAPTSEG_ERR_HIP;
  }
  if (pl.p.splits > 1) {
    ConvParams q = pl.p;
    q.out = final_out;
    if (defer && mode == MODE_WGRAD) {   // the sum runs at adaptseg_splitk_flush(s)
      std::lock_guard<std::mutex> lk(g_pending_mu);
      g_pending[s].push_back(PendingSum{q, slab, mode});
      return ADAPTSEG_OK;
    }
    return splitk_sum(q, slab, mode, s);
  }
  return ADAPTSEG_OK;
}


// bf16 (RNE) copy of a finished fp32 output, for the paths whose kernels do not write one.
__global__ void bf16_out_copy_kernel(const float *__restrict__ y, __bf16 *__restrict__ yb, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    yb[i] = (__bf16)y[i];
}

// F32X3 maths: the pixel-interleaved term images [rows][3][C] of a finished fp32 output
__global__ void x3_out_copy_kernel(const float *__restrict__ y, __bf16 *__restrict__ yb, int64_t n, int C) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t h, m, l;
    split3_2(y[i], 0.f, h, m, l);
    const int64_t o = (i / C) * 3 * C + i % C;
    yb[o] = __builtin_bit_cast(__bf16, (uint16_t)h);
    yb[o + C] = __builtin_bit_cast(__bf16, (uint16_t)m);
    yb[o + 2 * C] = __builtin_bit_cast(__bf16, (uint16_t)l);
  }
}

// ... four channels per thread (C % 4 == 0, 16-B aligned y, 8-B aligned terms, < 2^31 float4):
// one float4 load, three 8-B stores (the kernel above: 2-B stores and a 64-bit division per
// element)
__global__ void __launch_bounds__(256) x3_out_copy4_kernel(const float4 *__restrict__ y, uint2 *__restrict__ yb,
                                                           uint32_t n4, int C4, FastDiv fd_c4) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += gridDim.x * blockDim.x) {
    const uint32_t pix = fdiv(i, fd_c4);
    const uint32_t cq = i - pix * C4;
    uint2 h, m, l;
    split3(y[i], h, m, l);
    uint2 *o = yb + pix * 3 * C4 + cq;
    o[0] = h;
    o[C4] = m;
    o[2 * C4] = l;
  }
}

// F32X3 output term images written by the GEMM epilogue / split-K reduce itself (the F32X3
// kernels: the staged and term-image ones) instead of by out_copy's pass over the finished fp32
// output: 8-B aligned images, N % 4 == 0, < 2^31 term elements (the epilogue's 32-bit offsets)
static bool terms_in_epilogue(const Plan &pl, const uint16_t *yb, int64_t n) {
  return yb && pl.fast && pl.x3 && pl.p.N % 4 == 0 && 3 * n < (1ll << 31) && !(reinterpret_cast<uintptr_t>(yb) & 7);
}

// The operand copy of a finished output [n / C][C] (the paths whose kernels do not write it): a
// bf16 RNE image, or the three term images under the F32X3 maths
static int out_copy(const float *y, uint16_t *yb, int64_t n, int C, hipStream_t s) {
  if (!yb || n == 0) return ADAPTSEG_OK;
  AS_CHECK_ARG(y, "conv: an operand copy needs the fp32 output on this path");
  const unsigned blocks = (unsigned)std::min<int64_t>(ceil_div(n, 256), 8192);
  if (copies_are_terms() && C % 4 == 0 && n / 4 < (1ll << 31) / 3 && aligned16(y) &&
      !(reinterpret_cast<uintptr_t>(yb) & 7))
    x3_out_copy4_kernel<<<(unsigned)std::min<int64_t>(ceil_div(n / 4, 256), 16384), 256, 0, s>>>(
        reinterpret_cast<const float4 *>(y), reinterpret_cast<uint2 *>(yb), (uint32_t)(n / 4), C / 4,
        make_fastdiv(C / 4));
  else if (copies_are_terms())
    x3_out_copy_kernel<<<blocks, 256, 0, s>>>(y, reinterpret_cast<__bf16 *>(yb), n, C);
  else
    bf16_out_copy_kernel<<<blocks, 256, 0, s>>>(y, reinterpret_cast<__bf16 *>(yb), n);
  AS_CHECK_LAUNCH("out_copy");
  return ADAPTSEG_OK;
}

// Thin convs (Cout <= 4) go to the vector-ALU kernels of conv_thin.hip.
bool use_thin(const adaptseg_conv_desc *d, int op) { return thin_eligible(d, op); }

// The plan's kernel reads only the operand copies of the _x forms (the fp32 operand may be
// NULL): the LDS-DMA kernels, and the register-staged bf16 forward (its ABF form); for the
// tap-GEMM (ASPP) products, its inner GEMM's forward / weight gradient on an LDS-DMA kernel.
static bool copy_only(const Plan &pl, const adaptseg_conv_desc *d, int op) {
  if (use_thin(d, op)) return false;
  if (tapgemm_eligible(d)) return tapgemm_copy_only(d, op);
  if (copies_are_terms()) return pl.fast && pl.x3 && pl.x3r_ok;   // x3r on the caller's terms
  return pl.g16 || (pl.bf16 && op == ADAPTSEG_CONV_FWD);
}

// Bytes of the weight pack the plan's kernel reads (0: none).
static size_t plan_wpack_bytes(const Plan &pl) {
  if (pl.mode == MODE_WGRAD) return 0;
  if (pl.x3) return x3_wpack_bytes(pl);
  if (pl.bf16) return bf16_wpack_bytes(pl);
  return 0;
}

// A caller-built weight pack for the plan (adaptseg_conv2d_wpack): its kernel then skips the
// per-call pack.  Ignored when the final plan reads none (a misaligned operand downgraded it).
static int attach_wpack(Plan &pl, const void *w_pack) {
  pl.wpack_ext = nullptr;
  if (!w_pack || plan_wpack_bytes(pl) == 0) return ADAPTSEG_OK;
  AS_CHECK_ARG((reinterpret_cast<uintptr_t>(w_pack) & 15) == 0, "conv: weight pack must be 16-byte aligned");
  pl.wpack_ext = w_pack;
  return ADAPTSEG_OK;
}

}  // namespace adaptseg

using namespace adaptseg;

extern "C" {

int adaptseg_conv2d_workspace_size(const adaptseg_conv_desc *d, int op, size_t *bytes) {
  AS_CHECK_ARG(bytes, "null bytes");
  Plan pl;
  int st = make_plan(d, op, pl);
  if (st) return st;
  size_t b = pl.slab_bytes;
  if (pl.fast) {  // an unaligned operand at launch time falls back to the generic kernel
    Plan g = pl;
    g.fast = false;
    set_splits(g);
    b = std::max(b, g.slab_bytes);
  }
  if (pl.x3r_ok && copies_are_terms()) {   // the plan with the caller's term images
    Plan t = pl;
    x3_terms_flags(t);
    set_splits(t);
    b = std::max(b, t.slab_bytes);
  }
  if (tapgemm_eligible(d)) b = std::max(b, tapgemm_workspace(d, op));
  if (use_thin(d, op)) b = std::max(b, thin_workspace(d, op));
  if (op == ADAPTSEG_CONV_BWD_WEIGHT) {
    // bias-gradient partials
    int per, splits;
    bias_grad_split(d->n * d->oh * d->ow, d->k, &per, &splits);
    b = std::max(b, (size_t)splits * d->k * sizeof(float));
  }
  *bytes = b;
  return ADAPTSEG_OK;
}

int adaptseg_conv2d_kernel_id(const adaptseg_conv_desc *d, int op, int *kernel_id, int *splits) {
  AS_CHECK_ARG(kernel_id && splits, "conv2d_kernel_id: null");
  Plan pl;
  int st = make_plan(d, op, pl);
  if (st) return st;
  // alignment-dependent downgrades are not known here; report the aligned choice
  if (use_thin(d, op)) {
    *kernel_id = thin_kernel_id(op);
    *splits = 1;
    return ADAPTSEG_OK;
  }
  if (tapgemm_eligible(d)) return tapgemm_kernel_id(d, op, kernel_id, splits);
  *kernel_id = ::adaptseg::kernel_id(pl, op);
  *splits = pl.p.splits;
  return ADAPTSEG_OK;
}

int adaptseg_conv2d_kernel_id_x(const adaptseg_conv_desc *d, int op, int with_copies, int *kernel_id, int *splits) {
  AS_CHECK_ARG(kernel_id && splits, "conv2d_kernel_id_x: null");
  if (!with_copies || use_thin(d, op) || tapgemm_eligible(d)) return adaptseg_conv2d_kernel_id(d, op, kernel_id, splits);
  Plan pl;
  int st = make_plan(d, op, pl);
  if (st) return st;
  pl.act_ext = pl.act_ext2 = d;   // any non-NULL: the plan with the caller's operand copies
  x3_terms(pl);
  *kernel_id = ::adaptseg::kernel_id(pl, op);
  *splits = pl.p.splits;
  return ADAPTSEG_OK;
}

// The products with an operand-BN kernel (adaptseg_operand_bn): the x3h forward (selector 86)
// and the register-staged F32X3 weight gradient (295), on a BN of at most kAbnMaxC channels
static bool abn_plan_ok(const Plan &pl, const adaptseg_conv_desc *d, int op) {
  if (d->c > kAbnMaxC || d->c % 4 || d->nseg != 1 || use_thin(d, op) || tapgemm_eligible(d)) return false;
  const int kid = ::adaptseg::kernel_id(pl, op);
  return (op == ADAPTSEG_CONV_FWD && kid == 86) || (op == ADAPTSEG_CONV_BWD_WEIGHT && kid == 295);
}

int adaptseg_conv2d_operand_bn_ok(const adaptseg_conv_desc *d, int op, int *ok) {
  AS_CHECK_ARG(ok, "conv2d_operand_bn_ok: null");
  *ok = 0;
  Plan pl;
  int st = make_plan(d, op, pl);
  if (st) return st;
  if (op != ADAPTSEG_CONV_FWD && op != ADAPTSEG_CONV_BWD_WEIGHT) return ADAPTSEG_OK;
  set_splits(pl);
  x3_terms(pl);
  *ok = abn_plan_ok(pl, d, op) ? 1 : 0;
  return ADAPTSEG_OK;
}

static void set_abn(ConvParams &p, const adaptseg_operand_bn *abn) {
  p.abn_m = abn->mean;
  p.abn_is = abn->invstd;
  p.abn_w = abn->weight;
  p.abn_b = abn->bias;
}

int adaptseg_conv2d_copy_operand_only(const adaptseg_conv_desc *d, int op, int *only) {
  AS_CHECK_ARG(only, "conv2d_copy_operand_only: null");
  *only = 0;
  Plan pl;
  int st = make_plan(d, op, pl);
  if (st) return st;
  // the conditions the _x entry points accept a NULL fp32 operand under (aligned operands)
  *only = copy_only(pl, d, op) ? 1 : 0;
  return ADAPTSEG_OK;
}

int adaptseg_conv2d_wpack_size(const adaptseg_conv_desc *d, int op, size_t *bytes) {
  AS_CHECK_ARG(bytes, "conv2d_wpack_size: null");
  *bytes = 0;
  Plan pl;
  int st = make_plan(d, op, pl);
  if (st) return st;
  if (use_thin(d, op) || tapgemm_eligible(d)) return ADAPTSEG_OK;
  *bytes = plan_wpack_bytes(pl);
  return ADAPTSEG_OK;
}

int adaptseg_conv2d_wpack(const adaptseg_conv_desc *d, int op, const float *const *w, void *pack, size_t bytes,
                          adaptseg_stream_t stream) {
  Plan pl;
  int st = make_plan(d, op, pl);
  if (st) return st;
  AS_CHECK_ARG(w && pack, "conv2d_wpack: null pointer");
  AS_CHECK_ARG((reinterpret_cast<uintptr_t>(pack) & 15) == 0, "conv2d_wpack: pack must be 16-byte aligned");
  const size_t need = (use_thin(d, op) || tapgemm_eligible(d)) ? 0 : plan_wpack_bytes(pl);
  AS_CHECK_ARG(need > 0, "conv2d_wpack: this product reads no weight pack (size 0)");
  AS_CHECK_ARG(bytes >= need, "conv2d_wpack: %zu bytes < %zu", bytes, need);
  for (int s = 0; s < d->nseg; ++s) {
    AS_CHECK_ARG(w[s], "conv2d_wpack: null weight %d", s);
    // the pack kernels read float4 weight rows (a misaligned weight's conv plan reads no pack)
    AS_CHECK_ARG(aligned16(w[s]), "conv2d_wpack: weight %d must be 16-byte aligned", s);
    pl.p.wt[s] = w[s];
  }
  const hipError_t e = pl.x3 ? prep_x3_wpack(pl, pack, as_stream(stream)) : prep_bf16_wpack(pl, pack, as_stream(stream));
  if (e != hipSuccess) {
    set_error("conv2d_wpack: %s", hipGetErrorString(e));
    return ADAPTSEG_ERR_HIP;
  }
  return ADAPTSEG_OK;
}

int adaptseg_conv2d_fwd(const adaptseg_conv_desc *d, const float *x, const float *const *w,
                        const float *const *bias, const float *res, float *y, int flags, void *ws,
                        size_t ws_bytes, adaptseg_stream_t stream) {
  return adaptseg_conv2d_fwd_x(d, x, nullptr, w, nullptr, bias, res, y, nullptr, flags, ws, ws_bytes, stream);
}

int adaptseg_conv2d_fwd_x(const adaptseg_conv_desc *d, const float *x, const uint16_t *x_bf16,
                          const float *const *w, const void *w_pack, const float *const *bias, const float *res,
                          float *y, uint16_t *y_bf16, int flags, void *ws, size_t ws_bytes,
                          adaptseg_stream_t stream) {
  Plan pl;
  int st = make_plan(d, ADAPTSEG_CONV_FWD, pl);
  if (st) return st;
  AS_CHECK_ARG((x || x_bf16) && w && (y || y_bf16), "conv fwd: null pointer");
  AS_CHECK_ARG(y || !(use_thin(d, ADAPTSEG_CONV_FWD) || tapgemm_eligible(d)),
               "conv fwd: this product needs the fp32 output (thin / tap-GEMM path)");
  AS_CHECK_ARG(y || !(flags & ADAPTSEG_EPI_ACCUMULATE), "conv fwd: ACCUMULATE needs the fp32 output");
  AS_CHECK_ARG(x || (copy_only(pl, d, ADAPTSEG_CONV_FWD) && x_bf16),
               "conv fwd: this product needs the fp32 input (no bf16-operand kernel for it)");
  AS_CHECK_ARG(!(flags & kEpiActGrad), "conv fwd: *_GRAD flags not valid");
  AS_CHECK_ARG(!((flags & ADAPTSEG_EPI_LEAKY) && (flags & ADAPTSEG_EPI_RELU)), "conv fwd: LEAKY and RELU");
  AS_CHECK_ARG(!(flags & ADAPTSEG_EPI_RESIDUAL) || res, "conv fwd: residual flag without res");
  for (int s = 0; s < d->nseg; ++s) AS_CHECK_ARG(w[s], "conv fwd: null weight %d", s);
  const int64_t ny = (int64_t)d->n * d->oh * d->ow * d->k;
  if (use_thin(d, ADAPTSEG_CONV_FWD) &&
      thin_fwd(d, x, w[0], bias ? bias[0] : nullptr, res, y, flags, as_stream(stream)) == ADAPTSEG_OK)
    return out_copy(y, y_bf16, ny, d->k, as_stream(stream));
  if (tapgemm_eligible(d) && aligned16(x) && segs_aligned(w, d->nseg)) {
    st = tapgemm_fwd(d, x, x_bf16, w, bias, res, y, flags, ws, ws_bytes, as_stream(stream));
    return st ? st : out_copy(y, y_bf16, ny, d->k, as_stream(stream));
  }
  ConvParams &p = pl.p;
  p.x = x;
  for (int s = 0; s < d->nseg; ++s) {
    AS_CHECK_ARG(w[s], "conv fwd: null weight %d", s);
    p.wt[s] = w[s];
    p.bias[s] = bias ? bias[s] : nullptr;
    if (reinterpret_cast<uintptr_t>(w[s]) & 15) pl.vb = pl.fast = false;
  }
  if (reinterpret_cast<uintptr_t>(x) & 15) pl.va = pl.fast = false;
  set_splits(pl);
  pl.act_ext = aligned16(x_bf16) ? x_bf16 : nullptr;
  x3_terms(pl);
  // a misaligned weight clears pl.fast and, in set_splits, the bf16-operand kernel: only that
  // kernel reads the copy, so a NULL x needs it to survive the alignment checks too
  AS_CHECK_ARG(x || (copy_only(pl, d, ADAPTSEG_CONV_FWD) && pl.act_ext),
               "conv fwd: x is NULL but the plan (after the alignment checks) needs the fp32 input");
  const bool terms = copies_are_terms();   // F32X3: term images of y (the epilogue's, or a pass after the GEMM)
  AS_CHECK_ARG(y || !terms, "conv fwd: under the F32X3 maths the output is fp32 (y_bf16 is its term images)");
  const bool fused = terms && terms_in_epilogue(pl, y_bf16, ny);
  p.out = y;
  p.outb = (terms && !fused) ? nullptr : reinterpret_cast<__bf16 *>(y_bf16);
  p.outb_terms = fused ? 1 : 0;
  p.res = res;
  p.flags = flags;
  st = attach_wpack(pl, w_pack);
  if (st) return st;
  st = run_plan(pl, MODE_FWD, ws, ws_bytes, as_stream(stream));
  return (st || !terms || fused) ? st : out_copy(y, y_bf16, ny, d->k, as_stream(stream));
}

int adaptseg_conv2d_bnstats_size(const adaptseg_conv_desc *d, size_t *bytes) {
  AS_CHECK_ARG(bytes, "conv2d_bnstats_size: null");
  int st = validate(d);
  if (st) return st;
  // the smallest row tile any forward config uses (128) bounds the tile count
  const int64_t m = (int64_t)d->n * d->oh * d->ow;
  const int64_t nt = ceil_div(m, 128);
  *bytes = (size_t)(nt + 2 * (int64_t)d->k * nt) * sizeof(float);
  return ADAPTSEG_OK;
}

int adaptseg_conv2d_bnstats_tiles(const adaptseg_conv_desc *d, int *ntiles) {
  return adaptseg_conv2d_bnstats_tiles_x(d, 0, ntiles);
}

int adaptseg_conv2d_bnstats_tiles_x(const adaptseg_conv_desc *d, int with_copy, int *ntiles) {
  AS_CHECK_ARG(ntiles, "conv2d_bnstats_tiles: null");
  *ntiles = 0;
  Plan pl;
  int st = make_plan(d, ADAPTSEG_CONV_FWD, pl);
  if (st) return st;
  if (tapgemm_eligible(d)) return ADAPTSEG_OK;
  if (with_copy) {
    pl.act_ext = d;   // any non-NULL: the plan with the caller's copy of x
    x3_terms(pl);
  }
  if (pl.fast && pl.p.splits == 1)
    *ntiles = (int)ceil_div(pl.p.M, plan_bm(pl));
  return ADAPTSEG_OK;
}

int adaptseg_conv2d_fwd_bnstats(const adaptseg_conv_desc *d, const float *x, const float *const *w, float *y,
                                float *stats, size_t stats_bytes, int *ntiles, void *ws, size_t ws_bytes,
                                adaptseg_stream_t stream) {
  return adaptseg_conv2d_fwd_bnstats_x(d, x, nullptr, w, nullptr, y, nullptr, stats, stats_bytes, ntiles, ws, ws_bytes,
                                       stream);
}

static int fwd_bnstats_impl(const adaptseg_conv_desc *d, const float *x, const uint16_t *x_bf16,
                            const float *const *w, const void *w_pack, float *y, uint16_t *y_bf16, float *stats,
                            size_t stats_bytes, int *ntiles, void *ws, size_t ws_bytes, adaptseg_stream_t stream,
                            const adaptseg_operand_bn *abn);

int adaptseg_conv2d_fwd_bnstats_x(const adaptseg_conv_desc *d, const float *x, const uint16_t *x_bf16,
                                  const float *const *w, const void *w_pack, float *y, uint16_t *y_bf16,
                                  float *stats, size_t stats_bytes, int *ntiles, void *ws, size_t ws_bytes,
                                  adaptseg_stream_t stream) {
  return fwd_bnstats_impl(d, x, x_bf16, w, w_pack, y, y_bf16, stats, stats_bytes, ntiles, ws, ws_bytes, stream,
                          nullptr);
}

int adaptseg_conv2d_fwd_bnstats_abn(const adaptseg_conv_desc *d, const float *x_pre, const adaptseg_operand_bn *abn,
                                    const float *const *w, const void *w_pack, float *y, float *stats,
                                    size_t stats_bytes, int *ntiles, void *ws, size_t ws_bytes,
                                    adaptseg_stream_t stream) {
  AS_CHECK_ARG(abn && abn->mean && abn->invstd && x_pre, "conv fwd_bnstats_abn: null operand BN / input");
  return fwd_bnstats_impl(d, x_pre, nullptr, w, w_pack, y, nullptr, stats, stats_bytes, ntiles, ws, ws_bytes, stream,
                          abn);
}

static int fwd_bnstats_impl(const adaptseg_conv_desc *d, const float *x, const uint16_t *x_bf16,
                            const float *const *w, const void *w_pack, float *y, uint16_t *y_bf16, float *stats,
                            size_t stats_bytes, int *ntiles, void *ws, size_t ws_bytes, adaptseg_stream_t stream,
                            const adaptseg_operand_bn *abn) {
  AS_CHECK_ARG(ntiles && stats, "conv fwd_bnstats: null stats / ntiles");
  *ntiles = 0;
  Plan pl;
  int st = make_plan(d, ADAPTSEG_CONV_FWD, pl);
  if (st) return st;
  AS_CHECK_ARG((x || x_bf16) && w && (y || y_bf16), "conv fwd_bnstats: null pointer");
  AS_CHECK_ARG(y || !tapgemm_eligible(d), "conv fwd_bnstats: this product needs the fp32 output");
  AS_CHECK_ARG(x || copy_only(pl, d, ADAPTSEG_CONV_FWD),
               "conv fwd_bnstats: this product needs the fp32 input (no bf16-operand kernel for it)");
  for (int s = 0; s < d->nseg; ++s) AS_CHECK_ARG(w[s], "conv fwd_bnstats: null weight %d", s);
  AS_CHECK_ARG(!abn || !tapgemm_eligible(d), "conv fwd_bnstats_abn: no operand-BN kernel for this product");
  if (tapgemm_eligible(d))  // the tap-GEMM path has no fused statistics: plain forward
    return adaptseg_conv2d_fwd_x(d, x, x_bf16, w, nullptr, nullptr, nullptr, y, y_bf16, 0, ws, ws_bytes, stream);
  ConvParams &p = pl.p;
  p.x = x;
  for (int s = 0; s < d->nseg; ++s) {
    p.wt[s] = w[s];
    if (reinterpret_cast<uintptr_t>(w[s]) & 15) pl.vb = pl.fast = false;
  }
  if (reinterpret_cast<uintptr_t>(x) & 15) pl.va = pl.fast = false;
  set_splits(pl);
  pl.act_ext = aligned16(x_bf16) ? x_bf16 : nullptr;
  x3_terms(pl);
  AS_CHECK_ARG(x || (copy_only(pl, d, ADAPTSEG_CONV_FWD) && pl.act_ext),
               "conv fwd_bnstats: x is NULL but the plan (after the alignment checks) needs the fp32 input");
  if (abn) {
    AS_CHECK_ARG(abn_plan_ok(pl, d, ADAPTSEG_CONV_FWD),
                 "conv fwd_bnstats_abn: no operand-BN kernel for this product (adaptseg_conv2d_operand_bn_ok)");
    set_abn(p, abn);
  }
  const bool terms = copies_are_terms();
  AS_CHECK_ARG(y || !terms, "conv fwd_bnstats: under the F32X3 maths the output is fp32");
  const int64_t nyb = (int64_t)d->n * d->oh * d->ow * d->k;
  const bool fused = terms && terms_in_epilogue(pl, y_bf16, nyb);
  p.out = y;
  p.outb = (terms && !fused) ? nullptr : reinterpret_cast<__bf16 *>(y_bf16);
  p.outb_terms = fused ? 1 : 0;
  p.flags = 0;
  if (pl.fast && p.splits == 1) {
    const int nt = (int)ceil_div(p.M, plan_bm(pl));
    if ((size_t)(nt + 2 * (int64_t)p.N * nt) * sizeof(float) <= stats_bytes) {
      p.stats = stats;
      p.stats_ntiles = nt;
      *ntiles = nt;
    }
  }
  st = attach_wpack(pl, w_pack);
  if (st) return st;
  st = run_plan(pl, MODE_FWD, ws, ws_bytes, as_stream(stream));
  return (st || !terms || fused) ? st : out_copy(y, y_bf16, nyb, d->k, as_stream(stream));
}

int adaptseg_conv2d_bwd_data(const adaptseg_conv_desc *d, const float *dy, const float *const *w,
                             const float *res, const float *aux, float *dx, int flags, void *ws,
                             size_t ws_bytes, adaptseg_stream_t stream) {
  return adaptseg_conv2d_bwd_data_x(d, dy, nullptr, w, nullptr, res, aux, dx, nullptr, flags, ws, ws_bytes, stream);
}

int adaptseg_conv2d_bwd_data_x(const adaptseg_conv_desc *d, const float *dy, const uint16_t *dy_bf16,
                               const float *const *w, const void *w_pack, const float *res, const float *aux,
                               float *dx, uint16_t *dx_bf16, int flags, void *ws, size_t ws_bytes,
                               adaptseg_stream_t stream) {
  AS_CHECK_ARG(dx, "conv bwd_data: null dx (bf16-only outputs: adaptseg_conv2d_bwd_data_xg)");
  return adaptseg_conv2d_bwd_data_xg(d, dy, dy_bf16, w, w_pack, res, nullptr, nullptr, aux, dx, dx_bf16, flags, ws,
                                     ws_bytes, stream);
}

}  // extern "C"

namespace adaptseg {

// Fused BN backward sums: the row tiles of the data-gradient plan (0: it cannot fuse them — a
// thin / tap-GEMM / per-element / split-K / stride-2 product)
static int bnsum_plan_tiles(const Plan &pl, const adaptseg_conv_desc *d) {
  if (use_thin(d, ADAPTSEG_CONV_BWD_DATA) || tapgemm_eligible(d)) return 0;
  if (!pl.fast || pl.s2 || pl.p.splits != 1 || pl.g16) return 0;   // (g16: compiled out, igemm_epilogue)
  return (int)ceil_div(pl.p.M, plan_bm(pl));
}

// adaptseg_conv2d_bwd_data_xg, and with bs the fused BN backward sums where the final plan can
// produce them (*bs_tiles = its row tiles, else 0)
static int bwd_data_impl(const adaptseg_conv_desc *d, const float *dy, const uint16_t *dy_bf16,
                         const float *const *w, const void *w_pack, const float *res, const uint16_t *res_bf16,
                         const uint32_t *res_bits, const float *aux, float *dx, uint16_t *dx_bf16, int flags, void *ws,
                         size_t ws_bytes, adaptseg_stream_t stream, const adaptseg_bnsum_desc *bs, int *bs_tiles) {
  Plan pl;
  int st = make_plan(d, ADAPTSEG_CONV_BWD_DATA, pl);
  if (st) return st;
  AS_CHECK_ARG((dy || dy_bf16) && w && (dx || dx_bf16), "conv bwd_data: null pointer");
  AS_CHECK_ARG(!(res && res_bf16), "conv bwd_data: one residual pointer");
  // bf16 gradient storage (BF16 maths): the residual and / or the output as bf16 tensors
  const bool gb = res_bf16 || !dx;
  AS_CHECK_ARG(!gb || !copies_are_terms(), "conv bwd_data: bf16 gradient storage needs the BF16 conv maths");
  AS_CHECK_ARG(!gb || !(use_thin(d, ADAPTSEG_CONV_BWD_DATA) || tapgemm_eligible(d)),
               "conv bwd_data: the thin / tap-GEMM products take fp32 gradients only");
  AS_CHECK_ARG(!res_bf16 || aligned16(res_bf16), "conv bwd_data: res_bf16 must be 16-byte aligned");
  AS_CHECK_ARG(!res_bits || (d->c % 32 == 0 && !(use_thin(d, ADAPTSEG_CONV_BWD_DATA) || tapgemm_eligible(d))),
               "conv bwd_data: a residual mask bitmap needs Cin %% 32 == 0 and the implicit-GEMM path");
  AS_CHECK_ARG(dy || copy_only(pl, d, ADAPTSEG_CONV_BWD_DATA),
               "conv bwd_data: this product needs the fp32 dY (no bf16-operand kernel for it)");
  AS_CHECK_ARG(!(flags & (ADAPTSEG_EPI_LEAKY | ADAPTSEG_EPI_RELU)), "conv bwd_data: LEAKY/RELU not valid");
  AS_CHECK_ARG(!(flags & ADAPTSEG_EPI_RESIDUAL) || res || res_bf16, "conv bwd_data: residual flag without res");
  AS_CHECK_ARG(!(flags & kEpiActGrad) || aux, "conv bwd_data: *_GRAD without aux");
  AS_CHECK_ARG((flags & kEpiActGrad) != kEpiActGrad, "conv bwd_data: LEAKY_GRAD and RELU_GRAD");
  for (int s = 0; s < d->nseg; ++s) AS_CHECK_ARG(w[s], "conv bwd_data: null weight %d", s);
  const int64_t nx = (int64_t)d->n * d->h * d->w * d->c;
  if (use_thin(d, ADAPTSEG_CONV_BWD_DATA) &&
      thin_dgrad(d, dy, w[0], res, aux, dx, flags, as_stream(stream)) == ADAPTSEG_OK)
    return out_copy(dx, dx_bf16, nx, d->c, as_stream(stream));
  if (tapgemm_eligible(d) && aligned16(dy) && aligned16(dx) && segs_aligned(w, d->nseg) &&
      (!res || aligned16(res)) && (!aux || aligned16(aux))) {
    st = tapgemm_bwd_data(d, dy, w, res, aux, dx, flags, ws, ws_bytes, as_stream(stream));
    return st ? st : out_copy(dx, dx_bf16, nx, d->c, as_stream(stream));
  }
  ConvParams &p = pl.p;
  p.dy = dy;
  for (int s = 0; s < d->nseg; ++s) {
    AS_CHECK_ARG(w[s], "conv bwd_data: null weight %d", s);
    p.wt[s] = w[s];
    if (reinterpret_cast<uintptr_t>(w[s]) & 15) pl.vb = pl.fast = false;
  }
  if (reinterpret_cast<uintptr_t>(dy) & 15) pl.va = pl.fast = false;
  set_splits(pl);
  pl.act_ext = aligned16(dy_bf16) ? dy_bf16 : nullptr;
  x3_terms(pl);
  AS_CHECK_ARG(dy || ((pl.g16 || pl.x3ext) && pl.act_ext),
               "conv bwd_data: dy is NULL but the plan (after the alignment checks) needs the fp32 dY");
  const bool terms = copies_are_terms();
  const bool fused = terms && terms_in_epilogue(pl, dx_bf16, nx);
  p.out = dx;
  p.outb = (terms && !fused) ? nullptr : reinterpret_cast<__bf16 *>(dx_bf16);
  p.outb_terms = fused ? 1 : 0;
  p.res = res;
  p.resb = reinterpret_cast<const __bf16 *>(res_bf16);
  p.resbits = res_bits;
  p.aux = aux;
  p.flags = flags;
  if (bs) {
    const int nt = bnsum_plan_tiles(pl, d);
    const bool xal = bs->x ? aligned16(bs->x) : !(reinterpret_cast<uintptr_t>(bs->x_bf16) & 7);
    const bool cal = aligned16(bs->mean) && aligned16(bs->invstd) && (!bs->weight || aligned16(bs->weight)) &&
                     (!bs->bias || aligned16(bs->bias));
    if (nt > 0 && xal && cal && d->c % 4 == 0 && (size_t)2 * d->c * nt * sizeof(float) <= bs->partial_bytes) {
      p.bs_part = bs->partial;
      p.bs_x = bs->x;
      p.bs_xb = reinterpret_cast<const __bf16 *>(bs->x_bf16);
      p.bs_mean = bs->mean;
      p.bs_is = bs->invstd;
      p.bs_w = bs->weight;
      p.bs_b = bs->bias;
      p.bs_bits = bs->bits;
      p.bs_mask = bs->mask;
      p.bs_ntiles = nt;
      *bs_tiles = nt;
    }
  }
  st = attach_wpack(pl, w_pack);
  if (st) return st;
  st = run_plan(pl, MODE_DGRAD, ws, ws_bytes, as_stream(stream));
  if (st && bs_tiles) *bs_tiles = 0;
  return (st || !terms || fused) ? st : out_copy(dx, dx_bf16, nx, d->c, as_stream(stream));
}

}  // namespace adaptseg

extern "C" {

int adaptseg_conv2d_bwd_data_xg(const adaptseg_conv_desc *d, const float *dy, const uint16_t *dy_bf16,
                                const float *const *w, const void *w_pack, const float *res, const uint16_t *res_bf16,
                                const uint32_t *res_bits, const float *aux, float *dx, uint16_t *dx_bf16, int flags,
                                void *ws, size_t ws_bytes, adaptseg_stream_t stream) {
  return bwd_data_impl(d, dy, dy_bf16, w, w_pack, res, res_bf16, res_bits, aux, dx, dx_bf16, flags, ws, ws_bytes,
                       stream, nullptr, nullptr);
}

int adaptseg_conv2d_bnsum_tiles(const adaptseg_conv_desc *d, int with_copy, int *ntiles) {
  AS_CHECK_ARG(ntiles, "conv2d_bnsum_tiles: null");
  *ntiles = 0;
  Plan pl;
  int st = make_plan(d, ADAPTSEG_CONV_BWD_DATA, pl);
  if (st) return st;
  if (with_copy) {
    pl.act_ext = d;   // any non-NULL: the plan with the caller's copy of dY
    x3_terms(pl);
  }
  *ntiles = bnsum_plan_tiles(pl, d);
  return ADAPTSEG_OK;
}

int adaptseg_conv2d_bwd_data_bnsum(const adaptseg_conv_desc *d, const float *dy, const uint16_t *dy_bf16,
                                   const float *const *w, const void *w_pack, const float *res,
                                   const uint16_t *res_bf16, const uint32_t *res_bits, float *dx, uint16_t *dx_bf16,
                                   int flags, const adaptseg_bnsum_desc *bs, int *ntiles, void *ws, size_t ws_bytes,
                                   adaptseg_stream_t stream) {
  AS_CHECK_ARG(bs && ntiles, "conv bwd_data_bnsum: null bnsum descriptor / ntiles");
  *ntiles = 0;
  AS_CHECK_ARG((bs->x != nullptr) != (bs->x_bf16 != nullptr), "conv bwd_data_bnsum: exactly one of x / x_bf16");
  AS_CHECK_ARG(bs->mean && bs->invstd && bs->partial, "conv bwd_data_bnsum: null mean / invstd / partial");
  AS_CHECK_ARG(bs->mask >= 0 && bs->mask <= 2, "conv bwd_data_bnsum: mask %d (0 none, 1 ReLU from x, 2 bitmap)",
               bs->mask);
  AS_CHECK_ARG(bs->mask != 2 || (bs->bits && d->c % 32 == 0),
               "conv bwd_data_bnsum: a bitmap mask needs bits and C %% 32 == 0");
  return bwd_data_impl(d, dy, dy_bf16, w, w_pack, res, res_bf16, res_bits, nullptr, dx, dx_bf16, flags, ws, ws_bytes,
                       stream, bs, ntiles);
}

int adaptseg_conv2d_bwd_weight(const adaptseg_conv_desc *d, const float *dy, const float *x,
                               float *const *dw, float *const *db, int flags, void *ws,
                               size_t ws_bytes, adaptseg_stream_t stream) {
  return adaptseg_conv2d_bwd_weight_x(d, dy, nullptr, x, nullptr, dw, db, flags, ws, ws_bytes, stream);
}

static int bwd_weight_impl(const adaptseg_conv_desc *d, const float *dy, const uint16_t *dy_bf16, const float *x,
                           const uint16_t *x_bf16, float *const *dw, float *const *db, int flags, void *ws,
                           size_t ws_bytes, adaptseg_stream_t stream, const adaptseg_operand_bn *abn);

int adaptseg_conv2d_bwd_weight_x(const adaptseg_conv_desc *d, const float *dy, const uint16_t *dy_bf16,
                                 const float *x, const uint16_t *x_bf16, float *const *dw, float *const *db,
                                 int flags, void *ws, size_t ws_bytes, adaptseg_stream_t stream) {
  return bwd_weight_impl(d, dy, dy_bf16, x, x_bf16, dw, db, flags, ws, ws_bytes, stream, nullptr);
}

int adaptseg_conv2d_bwd_weight_abn(const adaptseg_conv_desc *d, const float *dy, const float *x_pre,
                                   const adaptseg_operand_bn *abn, float *const *dw, int flags, void *ws,
                                   size_t ws_bytes, adaptseg_stream_t stream) {
  AS_CHECK_ARG(abn && abn->mean && abn->invstd && x_pre && dy, "conv bwd_weight_abn: null operand BN / operand");
  return bwd_weight_impl(d, dy, nullptr, x_pre, nullptr, dw, nullptr, flags, ws, ws_bytes, stream, abn);
}

static int bwd_weight_impl(const adaptseg_conv_desc *d, const float *dy, const uint16_t *dy_bf16, const float *x,
                           const uint16_t *x_bf16, float *const *dw, float *const *db, int flags, void *ws,
                           size_t ws_bytes, adaptseg_stream_t stream, const adaptseg_operand_bn *abn) {
  Plan pl;
  int st = make_plan(d, ADAPTSEG_CONV_BWD_WEIGHT, pl);
  if (st) return st;
  AS_CHECK_ARG((dy || dy_bf16) && (x || x_bf16) && dw, "conv bwd_weight: null pointer");
  AS_CHECK_ARG((dy && x) || (dy_bf16 && x_bf16 && copy_only(pl, d, ADAPTSEG_CONV_BWD_WEIGHT) && !db) ||
                   (tapgemm_eligible(d) && dy && x_bf16 && copy_only(pl, d, ADAPTSEG_CONV_BWD_WEIGHT)),
               "conv bwd_weight: this product needs the fp32 operands (no bf16-operand kernel / bias gradient)");
  for (int s = 0; s < d->nseg; ++s) AS_CHECK_ARG(dw[s], "conv bwd_weight: null dw %d", s);
  hipStream_t s = as_stream(stream);
  AS_CHECK_ARG(!abn || !(use_thin(d, ADAPTSEG_CONV_BWD_WEIGHT) || tapgemm_eligible(d)),
               "conv bwd_weight_abn: no operand-BN kernel for this product");
  int thin_st = ADAPTSEG_ERR_ARG;
  if (use_thin(d, ADAPTSEG_CONV_BWD_WEIGHT)) {
    thin_st = thin_wgrad(d, dy, x, dw[0], flags, ws, ws_bytes, s);
    if (thin_st != ADAPTSEG_OK && thin_st != ADAPTSEG_ERR_ARG) return thin_st;
  }
  if (thin_st == ADAPTSEG_OK) {
    st = ADAPTSEG_OK;
  } else if (tapgemm_eligible(d) && aligned16(x) && segs_aligned(dw, d->nseg)) {
    st = tapgemm_bwd_weight(d, dy, x, x_bf16, dw, flags, ws, ws_bytes, s);
  } else {
    ConvParams &p = pl.p;
    p.dy = dy;
    p.x = x;
    for (int g = 0; g < d->nseg; ++g) p.dw[g] = dw[g];
    if (reinterpret_cast<uintptr_t>(dy) & 15) pl.va = pl.fast = false;
    if (reinterpret_cast<uintptr_t>(x) & 15) pl.vb = pl.fast = false;
    set_splits(pl);
    if (aligned16(dy_bf16) && aligned16(x_bf16) && dy_bf16 && x_bf16) {  // both copies or none
      pl.act_ext = dy_bf16;
      pl.act_ext2 = x_bf16;
    }
    x3_terms(pl);
    AS_CHECK_ARG((dy && x) || ((pl.g16 || pl.x3ext) && pl.act_ext),
                 "conv bwd_weight: dy / x is NULL but the plan (after the alignment checks) needs the fp32 operands");
    if (abn) {
      AS_CHECK_ARG(abn_plan_ok(pl, d, ADAPTSEG_CONV_BWD_WEIGHT),
                   "conv bwd_weight_abn: no operand-BN kernel for this product (adaptseg_conv2d_operand_bn_ok)");
      set_abn(p, abn);
    }
    p.flags = flags & ADAPTSEG_EPI_ACCUMULATE;
    // a deferred sum keeps its slabs in ws until the flush: not with a bias gradient, whose
    // partial sums reuse the start of ws right after this GEMM
    bool any_db = false;
    for (int g = 0; db && g < d->nseg; ++g) any_db |= db[g] != nullptr;
    st = run_plan(pl, MODE_WGRAD, ws, ws_bytes, s, (flags & ADAPTSEG_WGRAD_DEFER_SUM) && !any_db);
  }
  if (st) return st;
  if (db) {
    bool any = false;
    BiasOut o;
    for (int g = 0; g < 4; ++g) o.db[g] = g < d->nseg ? db[g] : nullptr;
    for (int g = 0; g < d->nseg; ++g) any |= db[g] != nullptr;
    if (any) {
      int rows = d->n * d->oh * d->ow;
      int per, splits;
      bias_grad_split(rows, d->k, &per, &splits);
      size_t need = (size_t)splits * d->k * sizeof(float);
      if (!ws || ws_bytes < need) {
        set_error("conv bias grad: workspace too small");
        return ADAPTSEG_ERR_WORKSPACE;
      }
      float *partial = reinterpret_cast<float *>(ws);
      if (bias_grad_vec(dy, d->k))
        bias_grad_partial4_kernel<<<splits, 256, 0, s>>>(reinterpret_cast<const float4 *>(dy), rows, d->k / 4, per,
                                                         reinterpret_cast<float4 *>(partial));
      else
        bias_grad_partial_kernel<<<splits, 256, 0, s>>>(dy, rows, d->k, per, partial);
      AS_CHECK_LAUNCH("bias_grad_partial");
      bias_grad_final_kernel<<<(unsigned)ceil_div(d->k, 4), 256, 0, s>>>(
          partial, splits, d->k, o, d->nseg, (flags & ADAPTSEG_EPI_ACCUMULATE) ? 1 : 0);
      AS_CHECK_LAUNCH("bias_grad_final");
    }
  }
  return ADAPTSEG_OK;
}

int adaptseg_conv_set_math(int math) {
  AS_CHECK_ARG(math == ADAPTSEG_MATH_F32 || math == ADAPTSEG_MATH_BF16 || math == ADAPTSEG_MATH_BF16_WIDE ||
                   math == ADAPTSEG_MATH_F32X3 || math == ADAPTSEG_MATH_F32X3_PRESPLIT,
               "conv_set_math: bad math %d", math);
  g_conv_math.store(math);
  return ADAPTSEG_OK;
}

int adaptseg_conv_set_option(int option, int value) {
  if (option == ADAPTSEG_OPT_X3H) {
    AS_CHECK_ARG(value >= 0 && value <= 7, "conv_set_option: X3H must be 0..7");
    g_opt_x3h.store(value);
  } else if (option == ADAPTSEG_OPT_G16_WIDE) {
    AS_CHECK_ARG(value >= 0 && value <= 3, "conv_set_option: G16_WIDE must be 0..3");
    g_opt_g16_wide.store(value);
  } else {
    AS_CHECK_ARG(false, "conv_set_option: unknown option %d", option);
  }
  return ADAPTSEG_OK;
}

int adaptseg_conv_get_option(int option, int *value) {
  AS_CHECK_ARG(value, "conv_get_option: null");
  if (option == ADAPTSEG_OPT_X3H) *value = x3h_mode();
  else if (option == ADAPTSEG_OPT_G16_WIDE) *value = g16_wide_mode();
  else AS_CHECK_ARG(false, "conv_get_option: unknown option %d", option);
  return ADAPTSEG_OK;
}

int adaptseg_splitk_flush(adaptseg_stream_t stream) {
  const hipStream_t s = as_stream(stream);
  std::vector<PendingSum> v;
  {
    std::lock_guard<std::mutex> lk(g_pending_mu);
    auto it = g_pending.find(s);
    if (it != g_pending.end()) v.swap(it->second);
  }
  for (const PendingSum &e : v) {
    const int st = splitk_sum(e.q, e.slab, e.mode, s);
    if (st) return st;
  }
  return ADAPTSEG_OK;
}

int adaptseg_splitk_pending(adaptseg_stream_t stream, int *count) {
  AS_CHECK_ARG(count, "splitk_pending: null");
  std::lock_guard<std::mutex> lk(g_pending_mu);
  auto it = g_pending.find(as_stream(stream));
  *count = it == g_pending.end() ? 0 : (int)it->second.size();
  return ADAPTSEG_OK;
}

int adaptseg_conv_get_math(int *math) {
  AS_CHECK_ARG(math, "conv_get_math: null");
  *math = g_conv_math.load();
  return ADAPTSEG_OK;
}

int adaptseg_timing_enable(int enable, int selector) {
  std::lock_guard<std::mutex> lk(g_timing.mu);
  g_timing.enabled = enable != 0;
  g_timing.selector = selector;
  if (enable) g_timing.used = 0;  // disabling keeps the recorded launches readable
  return ADAPTSEG_OK;
}

// Create event pairs up front (outside a timed region): a pair created on demand inside one — the
// pool ran out when the timed steps launch the roofline kernel more often than the untimed
// all-kernel step did — cost milliseconds each (c4 with its term-image data gradient as the
// roofline kernel: 195 -> 347 ms per step, profiles/r5/vgg_terms_thr_ab.txt)
int adaptseg_timing_reserve(int64_t pairs) {
  AS_CHECK_ARG(pairs >= 0 && pairs <= (1 << 20), "timing_reserve: bad count %lld", (long long)pairs);
  std::lock_guard<std::mutex> lk(g_timing.mu);
  while ((int64_t)g_timing.events.size() < pairs) {
    if (!timing_grow()) {
      set_error("timing_reserve: hipEventCreate failed");
      return ADAPTSEG_ERR_HIP;
    }
  }
  return ADAPTSEG_OK;
}

int adaptseg_stream_create_cu_mask(int k, int d, adaptseg_stream_t *stream) {
  AS_CHECK_ARG(stream && d > 0 && k > 0 && k <= d, "stream_create_cu_mask: bad arguments (k=%d d=%d)", k, d);
  int dev = 0, ncu = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  if (e != hipSuccess) {
    set_error("stream_create_cu_mask: %s", hipGetErrorString(e));
    return ADAPTSEG_ERR_HIP;
  }
  std::vector<uint32_t> mask((size_t)(ncu + 31) / 32, 0u);
  for (int i = 0; i < ncu; ++i)
    if (i % d < k) mask[i / 32] |= 1u << (i % 32);
  hipStream_t s = nullptr;
  e = hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data());
  if (e != hipSuccess) {
    set_error("hipExtStreamCreateWithCUMask: %s", hipGetErrorString(e));
    return ADAPTSEG_ERR_HIP;
  }
  *stream = reinterpret_cast<adaptseg_stream_t>(s);
  return ADAPTSEG_OK;
}

int adaptseg_stream_destroy(adaptseg_stream_t stream) {
  hipError_t e = hipStreamDestroy(as_stream(stream));
  if (e != hipSuccess) {
    set_error("hipStreamDestroy: %s", hipGetErrorString(e));
    return ADAPTSEG_ERR_HIP;
  }
  return ADAPTSEG_OK;
}

int adaptseg_timing_enable_stream(int enable) {
  std::lock_guard<std::mutex> lk(g_timing.mu);
  g_timing.stream_too = enable != 0;
  return ADAPTSEG_OK;
}

int adaptseg_timing_read_id_stream(int kernel_id, double *total_ms, int64_t *launches) {
  AS_CHECK_ARG(total_ms && launches, "timing_read_id_stream: null");
  std::lock_guard<std::mutex> lk(g_timing.mu);
  double ms = 0;
  int64_t n = 0;
  for (size_t i = 0; i < g_timing.used; ++i) {
    if (g_timing.ids[i] != kernel_id || !g_timing.has_stream[i]) continue;
    float t = 0.f;
    if (hipEventElapsedTime(&t, g_timing.sevents[i].first, g_timing.sevents[i].second) != hipSuccess) {
      set_error("timing_read_id_stream: event query failed (synchronise first)");
      return ADAPTSEG_ERR_HIP;
    }
    ms += t;
    ++n;
  }
  *total_ms = ms;
  *launches = n;
  return ADAPTSEG_OK;
}

int adaptseg_timing_enable_mem(int enable) {
  std::lock_guard<std::mutex> lk(g_timing.mu);
  g_timing.mem_enabled = enable != 0;
  return ADAPTSEG_OK;
}

int adaptseg_timing_read_id(int kernel_id, double *total_ms, double *total_units, int64_t *launches) {
  AS_CHECK_ARG(total_ms && total_units && launches, "timing_read_id: null");
  std::lock_guard<std::mutex> lk(g_timing.mu);
  double ms = 0, un = 0;
  int64_t n = 0;
  for (size_t i = 0; i < g_timing.used; ++i) {
    if (g_timing.ids[i] != kernel_id) continue;
    float t = 0.f;
    if (hipEventElapsedTime(&t, g_timing.events[i].first, g_timing.events[i].second) != hipSuccess) {
      set_error("timing_read_id: event query failed (synchronise first)");
      return ADAPTSEG_ERR_HIP;
    }
    ms += t;
    un += g_timing.flops[i];
    ++n;
  }
  *total_ms = ms;
  *total_units = un;
  *launches = n;
  return ADAPTSEG_OK;
}

int adaptseg_timing_read(double *total_ms, double *total_flops, int64_t *launches) {
  AS_CHECK_ARG(total_ms && total_flops && launches, "timing_read: null");
  std::lock_guard<std::mutex> lk(g_timing.mu);
  double ms = 0, fl = 0;
  int64_t n = 0;
  for (size_t i = 0; i < g_timing.used; ++i) {
    if (g_timing.ids[i] < 0 || g_timing.ids[i] >= kTimingMemBase) continue;
    ++n;
    float t = 0.f;
    if (hipEventElapsedTime(&t, g_timing.events[i].first, g_timing.events[i].second) != hipSuccess) {
      set_error("timing_read: event query failed (synchronise first)");
      return ADAPTSEG_ERR_HIP;
    }
    ms += t;
    fl += g_timing.flops[i];
  }
  *total_ms = ms;
  *total_flops = fl;
  *launches = n;
  return ADAPTSEG_OK;
}

}  // extern "C"
