// gfx950 kernels for the batched UDE RK4 solve (forward + VJP).
//
// Hot path replaced: torchdiffeq.odeint(ode, z, t, method='rk4',
// options=dict(step_size=h)) at lib/VAE.py:137 with ode in {Fp, Fa, FaFp}
// (lib/models.py:109-265), and the autograd backward of lib/VAE.py:203.
//
// Execution model (one workgroup = 4 waves = one tile of TT=16 trajectories):
//  * every MLP layer is a small GEMM  out[o][t] = W[o][:] . in[t][:]  on
//    v_mfma_f32_16x16x4_f32 (exact fp32); the 16 trajectories are the MFMA N
//    dimension, output rows are split across the 4 waves (row tiles of 16);
//  * activations live in LDS as one [t][feature] record per trajectory; weights
//    stream from L2 in a pre-packed fragment order (one 16-B load per lane feeds
//    4 MFMAs);
//  * all 4 RK4 stages of every step run inside the launch; the training forward saves
//    the 4 stage inputs per step (3R floats each) and each stage's activation rows
//    (Model::ACT_STORED) for the backward, which reads them back instead of re-running
//    the forward and back-propagates through the 3/8-rule;
//  * the parameter gradient dW[o][i] = sum_{t,eval} g[t][o] in[t][i] is another
//    MFMA GEMM (K = trajectories) whose accumulators stay in each wave's registers
//    for the whole launch (the wave owns the rows it computed in the forward);
//    per-workgroup partials are summed by a separate deterministic pass;
//  * latent dims >= 3 have zero derivative (lib/models.py:144, :249), so they are
//    per-trajectory constants: their layer-0 contribution W0[:,static].x + b0 is
//    hoisted once per tile, and their weight gradient uses the per-trajectory sum
//    of layer-0 output gradients (one GEMM per tile).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <utility>
#include <type_traits>
#include "ude_model.h"

namespace ude {

typedef float f4 __attribute__((ext_vector_type(4)));

template <class Fn, int... I>
__device__ __forceinline__ void sfor_i(Fn&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class Fn>
__device__ __forceinline__ void sfor(Fn&& f) {
  sfor_i(f, std::make_integer_sequence<int, N>{});
}

__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f4 f4zero() { f4 z = {0.f, 0.f, 0.f, 0.f}; return z; }

// Workgroup barrier for LDS hand-offs.  __syncthreads()'s workgroup-scope fence waits for every
// outstanding memory operation of the wave (s_waitcnt vmcnt(0)), so each barrier of the stage
// loop drained the prefetch loads issued a stage ahead (backward) and the checkpoint /
// activation-row stores (forward), exposing their HBM latency at every phase.  The RK4 kernels
// hand data between waves only through LDS (global results are read by later launches), so their
// barriers fence the LDS address space only: in-flight global loads and stores cross them.
__device__ __forceinline__ void lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

struct KArgs {
  const float* pack;
  const float* y0;
  const unsigned char* sched;
  float* latent;
  float* ckpt;
  double* stats_slab;
  const float* dlatent;
  // side statistics of the solve (backward: read) and their cotangents (nullable: zero)
  const float* st_mean;       // 2 floats: mean beta, mean gamma (posterior loc, lib/models.py:152-156)
  const float* st_std;        // 2 floats: unbiased std (posterior scale)
  const float* st_norm;       // 1 float: |Fa| (torch.norm(torch.stack(tracker)), lib/VAE.py:180)
  const float* d_mean;
  const float* d_std;
  const float* d_norm;
  float* dy0;
  float* slab;
  int n_traj, n_steps, n_out, n_tiles;
  float fa_w;
  unsigned long long* prof;   // diagnostic builds only (-DUDE_PROFILE): per-segment cycle sums
  float* g0buf;               // backward: per-trajectory layer-0 gradient sums [tile][K0][16]
  const float* eslab;         // BAYES backward: the eps stream in slab order, [eval][SLAB_TOTAL]
  const float* dlat_sir;      // backward: the compact S, I, R cotangent (T, N, R, 3) when dlatent is
                              // null (its dims >= 3 all zero); exactly one of the two is set
  const float* dec_pack;      // DEC forward: decoder fragments + bias (Model::DEC_PACK floats)
  float* yhat;                // DEC forward: (T, N, R) decoder outputs, written instead of the latent
  double* reg_slab;           // DEC forward: per-workgroup latent_init_loss partial sums
  float* ckpt_final;          // DEC training forward: the final-state block (ckpt + ckpt_final_off)
  float* gst;                 // GST backward: layer-output gradient rows [tile][step][stage][16][ACT_A4]
  // forward: the statistics finalised in the kernel by its last workgroup (ctl != nullptr; the
  // separate ude_stats_finalize_kernel otherwise)
  unsigned int* ctl;          // arrival counter, zero on entry, left zero
  float* o_mean;              // 2 floats
  float* o_std;               // 2 floats
  float* o_norm;              // 1 float
  double* o_sums;             // 5 doubles: sum beta, sum gamma, sum beta^2, sum gamma^2, sum Fa^2 (nullable)
  float* o_reg;               // DEC: latent_init_loss (1 float)
  double n_eval;              // 4 n_steps N R: the number of recorded rates per statistic
};

// latent_init_loss summand (lib/train_functions.py:116-126): |x| where x < 0, |1 - x| where x > 1
__device__ __forceinline__ float reg_term(float v) {
  return (v < 0.f ? fabsf(v) : 0.f) + (v > 1.f ? fabsf(1.f - v) : 0.f);
}

// Timing ablations for a diagnostic build (-DUDE_ABL=n, tools/ablate.py): component n of the
// small-record backward is skipped (results are wrong; only the kernel time is read).
#ifndef UDE_ABL
#define UDE_ABL 0
#endif
// Measured-off A/B variants of rounds 3-5 (two interleaved accumulation chains, early activation-row
// stores, row-mapped latent outputs, raised critical-path priority; round 5: input-gradient fragments
// a phase earlier, interleaved static hoist, tail time sums with fewer round trips, forward copy-wave
// priority, more static-gradient chunks) were removed from the tree: profiles/r04/ab_*.log and
// profiles/r05/ab_*.txt hold their measurements.

// In-kernel cycle stamps for a diagnostic build (-DUDE_PROFILE): wave-uniform
// s_memtime deltas accumulated per segment; compiled out otherwise.
constexpr int NPROF = 28;
constexpr int PROF_FWD_SLOT = 4096;          // the training forward's rows start at workgroup slot 4096
struct Prof {
  unsigned long long acc[NPROF];
  unsigned long long last;
};
#ifdef UDE_PROFILE
#define UDE_STAMP(pf, seg)                                                    \
  do {                                                                        \
    if (pf) {                                                                 \
      __builtin_amdgcn_sched_barrier(0);                                      \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime();             \
      __builtin_amdgcn_sched_barrier(0);                                      \
      (pf)->acc[seg] += t_ - (pf)->last;                                      \
      (pf)->last = t_;                                                        \
    }                                                                         \
  } while (0)
#else
#define UDE_STAMP(pf, seg) do { } while (0)
#endif

// Sum over the 16 lanes of a DPP row -- the 16 trajectories t = lane & 15 of a tile row -- by four
// DPP adds (quad_perm lane ^ 1, lane ^ 2, row_half_mirror, row_mirror): the association of the xor
// butterfly, so bitwise the same sums, without the LDS-crossbar ds_bpermute round trips of
// __shfl_xor (4 dependent LDS latencies per reduction).  Every lane of the row holds the sum.
// (state49 bwd 1.83 -> 1.72 ms, gradients bit-identical: profiles/r05/ab_dpp.txt)
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_mov<0xB1>(v);      // quad_perm [1, 0, 3, 2]
  v += dpp_mov<0x4E>(v);      // quad_perm [2, 3, 0, 1]
  v += dpp_mov<0x141>(v);     // row_half_mirror
  v += dpp_mov<0x140>(v);     // row_mirror
  return v;
}

// The step / output schedule (dt, the output CSR) is read every stage.  It is wave-uniform and
// read-only, so it is read through the constant address space: scalar loads (s_load, scalar
// cache) that count only in lgkmcnt.  A generic pointer compiled to FLAT loads, which count in
// vmcnt as well, so every schedule read waited for all of the wave's in-flight global stores
// (the forward's checkpoint and activation rows) and prefetch loads.
typedef const __attribute__((address_space(4))) float* SchedF;
typedef const __attribute__((address_space(4))) int* SchedI;
struct Sched {
  SchedF dt;
  SchedI out_start;
  SchedI out_j;
  SchedI out_mode;
  SchedF out_slope;
  __device__ Sched(const unsigned char* base, int n_steps, int n_out) {
    dt = (SchedF)base;
    out_start = (SchedI)(dt + n_steps);
    out_j = out_start + n_steps + 1;
    out_mode = out_j + n_out;
    out_slope = (SchedF)(out_mode + n_out);
  }
};

// Packed weights are read through a buffer resource (SGPR descriptor): every
// fragment load is `voffset = lane*16` + a compile-time scalar offset, so no
// per-tile 64-bit lane addresses are materialised (they were hoisted out of the
// step loop and spilled).
typedef __amdgpu_buffer_rsrc_t Rsrc;
__device__ __forceinline__ Rsrc make_rsrc(const float* p, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), 0, bytes, 0x00020000);
}
__device__ __forceinline__ f4 ldw(Rsrc rs, int voff_bytes, int soff_bytes) {
  return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff_bytes, soff_bytes, 0));
}

// One 16-row tile of  C[o][t] += sum_k A[o][k] * B[t][k]  with K = KP (multiple of 16).
// A: packed fragments at float offset WOFF of the pack ([KP/16][64][4] for this tile);
// B: the per-trajectory LDS record, lane group g reading features [g*KP/4, (g+1)*KP/4).
template <int KP, int WOFF>
__device__ __forceinline__ f4 gemm_tile(Rsrc rs, const float* bp, int lane, f4 acc) {
  constexpr int KQ = KP / 4;
  constexpr int NQ = KP / 16;
  const float* b = bp + (lane >> 4) * KQ;
  // every A fragment of the tile is issued before the first MFMA (the scheduler
  // otherwise serialises load -> wait -> 4 MFMAs, paying the L2 latency per quad)
  f4 a[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) a[q] = ldw(rs, lane * 16, (WOFF + q * 256) * 4);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const f4 x = *reinterpret_cast<const f4*>(b + 4 * q);
    acc = mfma4(a[q][0], x[0], acc);
    acc = mfma4(a[q][1], x[1], acc);
    acc = mfma4(a[q][2], x[2], acc);
    acc = mfma4(a[q][3], x[3], acc);
  }
  return acc;
}

// As gemm_tile with the A fragments in flight QC quads at a time (4 QC VGPRs): for a GEMM outside
// the stage loop's critical path in a kernel at its register limit (the DEC forward's decoder).
template <int KP, int WOFF, int QC>
__device__ __forceinline__ f4 gemm_tile_lean(Rsrc rs, const float* bp, int lane, f4 acc) {
  constexpr int KQ = KP / 4, NQ = KP / 16;
  const float* b = bp + (lane >> 4) * KQ;
#pragma unroll
  for (int q0 = 0; q0 < NQ; q0 += QC) {
    f4 a[QC];
#pragma unroll
    for (int q = 0; q < QC; ++q)
      if (q0 + q < NQ) a[q] = ldw(rs, lane * 16, (WOFF + (q0 + q) * 256) * 4);
#pragma unroll
    for (int q = 0; q < QC; ++q) {
      if (q0 + q < NQ) {
        const f4 x = *reinterpret_cast<const f4*>(b + 4 * (q0 + q));
        acc = mfma4(a[q][0], x[0], acc);
        acc = mfma4(a[q][1], x[1], acc);
        acc = mfma4(a[q][2], x[2], acc);
        acc = mfma4(a[q][3], x[3], acc);
      }
    }
  }
  return acc;
}

// Split form: issue a tile's fragments into a caller array (so several tiles, or a
// whole phase, can be in flight before the first MFMA), then run the MFMA chain.
template <int KP, int WOFF>
__device__ __forceinline__ void load_frags(Rsrc rs, int lane, f4* fr) {
#pragma unroll
  for (int q = 0; q < KP / 16; ++q) fr[q] = ldw(rs, lane * 16, (WOFF + q * 256) * 4);
}
template <int KP>
__device__ __forceinline__ f4 mma_frags(const f4* fr, const float* bp, int lane, f4 acc) {
  constexpr int KQ = KP / 4;
  const float* b = bp + (lane >> 4) * KQ;
#pragma unroll
  for (int q = 0; q < KP / 16; ++q) {
    const f4 x = *reinterpret_cast<const f4*>(b + 4 * q);
    acc = mfma4(fr[q][0], x[0], acc);
    acc = mfma4(fr[q][1], x[1], acc);
    acc = mfma4(fr[q][2], x[2], acc);
    acc = mfma4(fr[q][3], x[3], acc);
  }
  return acc;
}

// ELU (alpha 1).  expm1 is evaluated unconditionally on min(x, 0) and selected,
// so the compiler emits straight-line code instead of a divergent branch per value.
// (libm expm1f: torch's expm1-grade accuracy; the adaptive dopri5 step control is
// sensitive to the last bits of the RHS, measured: a 1-ulp-of-1 exp2 variant moves its
// evaluation points enough to shift the side statistics by 2e-3.)
__device__ __forceinline__ float elu1(float x) {
  const float e = expm1f(fminf(x, 0.f));
  return x > 0.f ? x : e;
}

template <class M, int NZ_>
using C1Arr = f4[NZ_ > 0 ? NZ_ : 1];

// Input-gradient (dX) fragments of wave W at depth d: [XQ(W, d)] quads in tile order.
template <class M, int W, int d>
__device__ __forceinline__ void load_x_frags(Rsrc rs, int lane, f4* fx) {
  if constexpr (d == 0 && M::SPLITX0) {
    // wave W's K quads qq = W (mod WAVES) of every layer-0 input tile m (merged nets, P first)
    constexpr int PQ = M::HAS_P ? M::kout(0, 0) / 16 : 0;
    sfor<M::XT(0)>([&](auto mm) {
      constexpr int m = decltype(mm)::value;
      sfor<M::x0q_w(W)>([&](auto jj) {
        constexpr int j = decltype(jj)::value, qq = W + j * WAVES;
        constexpr int net = qq < PQ ? 0 : 1, q = qq < PQ ? qq : qq - PQ;
        fx[m * M::x0q_w(W) + j] =
            ldw(rs, lane * 16, (M::wt_off(net, 0) + m * (M::kout(net, 0) / 16) * 256 + q * 256) * 4);
      });
    });
    return;
  }
  sfor<M::XT(d)>([&](auto mm) {
    constexpr int m = decltype(mm)::value;
    if constexpr (M::xowner(d, m) == W) {
      constexpr int q0 = M::xq_before(W, d, m);
      if constexpr (d == 0) {
        if constexpr (M::HAS_P)
          load_frags<M::kout(0, 0), M::wt_off(0, 0) + m * (M::kout(0, 0) / 16) * 256>(rs, lane, fx + q0);
        if constexpr (M::HAS_A)
          load_frags<M::kout(1, 0), M::wt_off(1, 0) + m * (M::kout(1, 0) / 16) * 256>(
              rs, lane, fx + q0 + (M::HAS_P ? M::kout(0, 0) / 16 : 0));
      } else {
        constexpr int net = M::xnet(d, m), rt = M::xrt(d, m);
        load_frags<M::kout(net, d), M::wt_off(net, d) + rt * (M::kout(net, d) / 16) * 256>(rs, lane, fx + q0);
      }
    }
  });
}

// Layer 0 of a record with at most 4 dynamic features (R = 1: S, I, R) and the static ones hoisted: every
// K step but the first multiplies padding, so the phase runs ONE MFMA per output tile with lane (o, g)
// holding W[o][g] and feature g instead of KP / 4 -- the same non-zero products added in the same order
// (the padded steps add exact zeros), so bitwise the same layer output.  With packo below: M1 FaFp step
// 7.50 -> 7.34 ms, gradients bitwise equal (profiles/r06/ab_pack_r1/).
template <class M>
constexpr bool pack0() { return M::HOIST && M::F <= 4 && M::F16 == 16; }
// ... for the waves that own at least two layer-0 tiles: with one tile per wave (Fp [32, 32]) the packed
// phase measured 1% slower (fwd 1.507 -> 1.522 ms, profiles/r06/ab_pack_r1/ab_fp32_4way.txt)
template <class M, int W>
constexpr bool pack0_w() { return pack0<M>() && M::NZ(W) >= 2; }
// The same for the input gradient of an output layer with at most 4 outputs (R = 1: the 2 rates, the 3
// Fa components): K = the 16-padded outputs, one MFMA per input tile with lane (h, g) holding W[g][h]
// and dZ[g] (register-resident weights only: the packed values are formed once per launch).
template <class M>
constexpr bool packo(int net, int d) {
  return M::has(net, d) && d > 0 && d == M::nl(net) - 1 && M::kout(net, d) == 16 && M::out_dim(net, d) <= 4;
}

// Register-resident weights (Model::WREG): every fragment / bias quad wave W reads in the
// forward (and, BWD, the input-gradient fragments), loaded once per launch.
struct NoWRegs {
  static constexpr bool ON = false;
  f4 wf[1], wb[1], wx[1];
};
template <class M, int W, bool BWD, bool NEED_F_ = !BWD || !M::ACT_STORED, bool FORCE = false>
struct WRegs {
  static constexpr bool ON = M::WREG || FORCE;
  static constexpr bool NEED_F = NEED_F_;   // a stored-activation RK4 backward never runs the forward
  static constexpr int NF = (ON && NEED_F) ? M::WF_Q(W) : 0, NB = (ON && NEED_F) ? M::WB_Q(W) : 0;
  static constexpr int NX = (ON && BWD) ? M::WX_Q(W) : 0;
  static constexpr int NP0 = (ON && NEED_F && pack0_w<M, W>()) ? M::NZ(W) : 0;
  // packo: the wave's output-layer input-gradient tiles in (d, m) order
  static constexpr int po_index(int d, int m) {
    int c = 0;
    for (int e = 0; e < M::D; ++e)
      for (int j = 0; j < M::XT(e); ++j) {
        if (e == d && j == m) return c;
        if (M::xowner(e, j) == W && packo<M>(M::xnet(e, j), e)) ++c;
      }
    return c;
  }
  static constexpr int NPO = (ON && BWD) ? po_index(M::D, 0) : 0;
  f4 wf[NF > 0 ? NF : 1], wb[NB > 0 ? NB : 1], wx[NX > 0 ? NX : 1];
  float w0[NP0 > 0 ? NP0 : 1];              // pack0: lane (o, g)'s layer-0 weight W[o][g]
  float wo[NPO > 0 ? NPO : 1];              // packo: lane (h, g)'s output-layer weight W[g][h]
  __device__ __forceinline__ void load(Rsrc rs, int lane, bool wait = true) {
    if constexpr (ON) {
      const int g = lane >> 4;
      sfor<M::D>([&](auto dd) {
        constexpr int d = decltype(dd)::value;
        if constexpr (NEED_F) sfor<M::FT(d)>([&](auto kk) {
          constexpr int k = decltype(kk)::value;
          if constexpr (M::fowner(d, k) == W) {
            constexpr int net = M::fnet(d, k), rt = M::frt(d, k), KP = M::kin(net, d);
            load_frags<KP, M::wf_off(net, d) + rt * (KP / 16) * 256>(rs, lane,
                                                                     wf + M::fq_base(W, d) + M::fq_before(W, d, k));
            if constexpr (M::has_bias(d))
              wb[M::nb_base(W, d) + M::nb_before(W, d, k)] = ldw(rs, g * 16, (M::b_off(net, d) + rt * 16) * 4);
          }
        });
        if constexpr (BWD) load_x_frags<M, W, d>(rs, lane, wx + M::xq_base(W, d));
      });
      // wait for the fragments here, once: the loop-carried wait analysis otherwise keeps them
      // "pending" at the step loop's head and puts a vmcnt(0) before the first MFMA of every
      // stage, which also drains the loads prefetched a stage ahead (s_waitcnt vmcnt(0))
      if (wait) __builtin_amdgcn_s_waitcnt(0x0F70);
      if constexpr (NP0 > 0) {
        // lane (o, g) takes element g of lane (o, 0)'s fragment quad (W[o][0..3]), once per launch
        sfor<M::FT(0)>([&](auto kk) {
          constexpr int k = decltype(kk)::value;
          if constexpr (M::fowner(0, k) == W) {
            const f4 q = wf[M::fq_base(W, 0) + M::fq_before(W, 0, k)];
            const int src = lane & 15;
            const float v0 = __shfl(q[0], src, 64), v1 = __shfl(q[1], src, 64);
            const float v2 = __shfl(q[2], src, 64), v3 = __shfl(q[3], src, 64);
            w0[M::nz_before(W, k)] = g == 0 ? v0 : (g == 1 ? v1 : (g == 2 ? v2 : v3));
          }
        });
      }
      if constexpr (NPO > 0) {
        sfor<M::D>([&](auto dd) {
          constexpr int d = decltype(dd)::value;
          if constexpr (d > 0) sfor<M::XT(d)>([&](auto mm) {
            constexpr int m = decltype(mm)::value;
            if constexpr (M::xowner(d, m) == W && packo<M>(M::xnet(d, m), d)) {
              // K = 16 outputs: one quad per tile, lane (h, g) holds W[4 g + e][h]
              const f4 q = wx[M::xq_base(W, d) + M::xq_before(W, d, m)];
              const int src = lane & 15;
              const float v0 = __shfl(q[0], src, 64), v1 = __shfl(q[1], src, 64);
              const float v2 = __shfl(q[2], src, 64), v3 = __shfl(q[3], src, 64);
              wo[po_index(d, m)] = g == 0 ? v0 : (g == 1 ? v1 : (g == 2 ? v2 : v3));
            }
          });
        });
      }
    }
  }
};

// Forward pass of both MLPs for the stage input held in the record's Y slot.
// Leaves post-activation outputs of every layer in the record (the final
// layers' raw outputs: P-net pre-|.| rates q, A-net Fa).  Ends on a barrier.
struct NoHook {
  template <class D>
  __device__ __forceinline__ void operator()(D) const {}
};

// `hook(integral_constant<d>)` runs right after phase d's weight loads are issued
// (used by the backward to start HBM loads early without holding registers long).
template <class M, int W, int SR, class WR = NoWRegs, class Hook = NoHook>
__device__ __forceinline__ void mlp_forward(Rsrc rs, float* lds, const f4* c1, int lane, const WR& wr = WR{},
                                            Prof* pf = nullptr, const Hook& hook = Hook{}) {
  constexpr bool RW = WR::ON;
  const int t = lane & 15, g = lane >> 4;
  float* rec = lds + t * SR;
  sfor<M::D>([&](auto dd) {
    constexpr int d = decltype(dd)::value;
    constexpr int NF = M::FQ(W, d);
    // all of this wave's weight fragments (and biases) for the phase are in flight
    // before its first MFMA -- unless they would not fit next to the working set (the Bayesian
    // state model's layer 0, K = 416: 208 VGPRs, spilled at the forward's 256): then chunk by chunk
    constexpr bool CHUNK_A = !RW && NF > 24;
    constexpr bool P0 = d == 0 && pack0_w<M, W>();
    f4 fr[(NF > 0 && !RW && !CHUNK_A) ? NF : 1], bias[(M::FT(d) > 0 && !RW) ? M::FT(d) : 1];
    float w0s[(P0 && !RW && M::NZ(W) > 0) ? M::NZ(W) : 1];
    if constexpr (!RW) {
      sfor<M::FT(d)>([&](auto kk) {
        constexpr int k = decltype(kk)::value;
        if constexpr (M::fowner(d, k) == W) {
          constexpr int net = M::fnet(d, k), rt = M::frt(d, k), KP = M::kin(net, d);
          if constexpr (P0) {
            // W[o][g]: element g of lane (o, 0)'s fragment quad
            w0s[M::nz_before(W, k)] = __builtin_bit_cast(
                float, __builtin_amdgcn_raw_buffer_load_b32(rs, ((lane & 15) * 4 + g) * 4,
                                                            (M::wf_off(net, d) + rt * (KP / 16) * 256) * 4, 0));
          } else if constexpr (!CHUNK_A) {
            load_frags<KP, M::wf_off(net, d) + rt * (KP / 16) * 256>(rs, lane, fr + M::fq_before(W, d, k));
          }
          if constexpr (M::has_bias(d)) bias[k] = ldw(rs, g * 16, (M::b_off(net, d) + rt * 16) * 4);
        }
      });
    }
    auto FR = [&](int i) -> f4 {
      if constexpr (RW) return wr.wf[M::fq_base(W, d) + i];
      else return fr[i];
    };
    hook(dd);
    __builtin_amdgcn_sched_barrier(0);
    f4 acc[M::FT(d) > 0 ? M::FT(d) : 1];
    sfor<M::FT(d)>([&](auto kk) {
      constexpr int k = decltype(kk)::value;
      if constexpr (M::fowner(d, k) == W) {
        if constexpr (d == 0 && M::HOIST) acc[k] = c1[M::nz_before(W, k)];
        else if constexpr (RW) acc[k] = wr.wb[M::nb_base(W, d) + M::nb_before(W, d, k)];
        else acc[k] = bias[k];
      }
    });
    if constexpr (P0) {
      // pack0: one MFMA per owned tile, lane (t, g) supplies feature g of trajectory t
      const float xg = g < M::F ? rec[M::Y_OFF + g] : 0.f;
      sfor<M::FT(d)>([&](auto kk) {
        constexpr int k = decltype(kk)::value;
        if constexpr (M::fowner(d, k) == W) {
          float wv;
          if constexpr (RW) wv = wr.w0[M::nz_before(W, k)];
          else wv = w0s[M::nz_before(W, k)];
          acc[k] = mfma4(wv, xg, acc[k]);
        }
      });
    }
    // the wave's tiles of one net share the B operand (the layer input): one LDS
    // read feeds every tile, and consecutive MFMAs go to different accumulators
    if constexpr (!P0) sfor<2>([&](auto nn) {
      constexpr int net = decltype(nn)::value;
      if constexpr (M::owns_f(W, d, net)) {
        constexpr int KP = M::kin(net, d);
        constexpr int inoff = d == 0 ? M::Y_OFF : M::act_off(net, d - 1);
        const float* b = rec + inoff + g * (KP / 4);
        // B quads are read in chunks of QB ahead of their MFMAs (one LDS wait per chunk)
        constexpr int NQ = KP / 16, QB = CHUNK_A ? 4 : 5;
        // CHUNK_A: the chunks' weight fragments double-buffered, chunk c + 1's loads in flight
        // during chunk c's MFMAs (fully unrolled: the buffer index is a constant)
        f4 fa[2][CHUNK_A ? M::FT(d) : 1][CHUNK_A ? QB : 1];
        auto load_chunk = [&](int bsel, int c0) {
          if constexpr (CHUNK_A)
            sfor<M::FT(d)>([&](auto kk) {
              constexpr int k = decltype(kk)::value;
              if constexpr (M::fowner(d, k) == W && M::fnet(d, k) == net) {
                constexpr int rt = M::frt(d, k);
#pragma unroll
                for (int q = c0; q < c0 + QB && q < NQ; ++q)
                  fa[bsel][k][q - c0] = ldw(rs, lane * 16, (M::wf_off(net, d) + rt * NQ * 256 + q * 256) * 4);
              }
            });
        };
        load_chunk(0, 0);
#pragma unroll
        for (int q0 = 0; q0 < NQ; q0 += QB) {
          f4 xb[QB];
          const int cb = (q0 / QB) & 1;
          if (q0 + QB < NQ) load_chunk(cb ^ 1, q0 + QB);
#pragma unroll
          for (int q = q0; q < q0 + QB && q < NQ; ++q) xb[q - q0] = *reinterpret_cast<const f4*>(b + 4 * q);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int q = q0; q < q0 + QB && q < NQ; ++q) {
            const f4 x = xb[q - q0];
#pragma unroll
            for (int e = 0; e < 4; ++e)
              sfor<M::FT(d)>([&](auto kk) {
                constexpr int k = decltype(kk)::value;
                if constexpr (M::fowner(d, k) == W && M::fnet(d, k) == net) {
                  f4 wq;
                  if constexpr (CHUNK_A) wq = fa[cb][CHUNK_A ? k : 0][CHUNK_A ? q - q0 : 0];
                  else wq = FR(M::fq_before(W, d, k) + q);
                  if constexpr (UDE_ABL == 13) acc[k][e] += x[e];
                  else acc[k] = mfma4(wq[e], x[e], acc[k]);
                }
              });
          }
        }
      }
    });
    sfor<M::FT(d)>([&](auto kk) {
      constexpr int k = decltype(kk)::value;
      if constexpr (M::fowner(d, k) == W) {
        constexpr int net = M::fnet(d, k), rt = M::frt(d, k);
        f4 a = acc[k];
        if constexpr (M::act(net, d)) {
          a[0] = elu1(a[0]); a[1] = elu1(a[1]);
          a[2] = elu1(a[2]); a[3] = elu1(a[3]);
        }
        *reinterpret_cast<f4*>(rec + M::act_off(net, d) + rt * 16 + g * 4) = a;
      }
    });
    lds_sync();
    UDE_STAMP(pf, 2 + d);
  });
}

// Static-feature hoist: c1[o][t] = b0[o] + sum_s W0[o][static s] * x_static[t][s].
template <class M, int W, int SR, int XOFF>
__device__ __forceinline__ void static_hoist(Rsrc rs, const float* lds, f4* c1, int lane) {
  if constexpr (M::HOIST) {
    const int t = lane & 15, g = lane >> 4;
    sfor<M::FT(0)>([&](auto kk) {
      constexpr int k = decltype(kk)::value;
      if constexpr (M::fowner(0, k) == W) {
        constexpr int net = M::fnet(0, k);
        constexpr int rt = M::frt(0, k);
        f4 acc = ldw(rs, g * 16, (M::b_off(net, 0) + rt * 16) * 4);
        acc = gemm_tile<M::S16, M::wsf_off(net) + rt * (M::S16 / 16) * 256>(rs, lds + t * SR + XOFF, lane, acc);
        c1[M::nz_before(W, k)] = acc;
      }
    });
    __builtin_amdgcn_s_waitcnt(0x0F70);   // once per tile (see WRegs::load)
  }
}

// Load the tile's static features (latent dims >= 3 of y0) into the record.
template <class M, int SR, int XOFF>
__device__ __forceinline__ void load_static(const float* __restrict__ y0, float* lds, int n0, int n_traj) {
  if constexpr (M::S > 0) {
    #pragma unroll 1
    for (int i = threadIdx.x; i < TT * M::S16; i += NTHREADS) {
      const int t = i / M::S16, s = i - t * M::S16;
      const int n = n0 + t;
      float v = 0.f;
      if (s < M::S && n < n_traj) {
        const int r = s / (M::L - 3), c = 3 + s - r * (M::L - 3);
        v = y0[((size_t)n * M::R + r) * M::L + c];
      }
      lds[t * SR + XOFF + s] = v;
    }
  }
}

// Forward tile start (L = 8), before the stage input: the record's static features from y0, CS loads in
// flight at a time, ahead of any global store of the tile (loads and stores count together in vmcnt, so a
// load issued behind pending stores waits for them to complete).
template <class M, int SR, int XOFF>
__device__ __forceinline__ void fwd_tile_static(const KArgs& A, float* lds, int n0) {
  // every load of the thread in flight at once (state49: 16; 4 at a time measured fwd 0.921 -> 0.909 ms
  // against this, profiles/r05/ab_tile_static.txt)
  constexpr int PS = (TT * M::S16 + NTHREADS - 1) / NTHREADS, CS = PS < 16 ? PS : 16;
  int tid = threadIdx.x;
  // thread-derived offsets formed here each tile, not hoisted into registers the stage loop needs
  asm volatile("" : "+v"(tid));
#pragma unroll
  for (int u0 = 0; u0 < PS; u0 += CS) {
    float sv[CS];
#pragma unroll
    for (int uu = 0; uu < CS; ++uu) {
      const int i = tid + (u0 + uu) * NTHREADS;
      const int t = i / M::S16, s = i - t * M::S16;
      const int n = n0 + t;
      float v = 0.f;
      if (u0 + uu < PS && i < TT * M::S16 && s < M::S && n < A.n_traj) {
        const int r = s / (M::L - 3), c = 3 + s - r * (M::L - 3);
        v = A.y0[((size_t)n * M::R + r) * M::L + c];
      }
      sv[uu] = v;
    }
#pragma unroll
    for (int uu = 0; uu < CS; ++uu) {
      const int i = tid + (u0 + uu) * NTHREADS;
      const int t = i / M::S16, s = i - t * M::S16;
      if (u0 + uu < PS && i < TT * M::S16) lds[t * SR + XOFF + s] = sv[uu];
    }
  }
}

// latent[0] and the static latent dims of every output time (zero derivative, carried unchanged:
// lib/models.py:144), from the record (stage input in the Y slot, static features at XOFF) after the
// tile-start barrier: stores only, row-mapped (consecutive lanes, consecutive 32-B (n, r) rows of the
// tile's contiguous (16, R, 8) latent block).  The per-output copy loop this replaces read y0 once per
// iteration behind its own pending stores (18% of the state49 training forward, tools/stage_profile.py).
template <class M, int SR, int XOFF>
__device__ __forceinline__ void fwd_tile_latent(const KArgs& A, const Sched& sc, const float* lds, int n0) {
  constexpr int NROW = TT * M::R, PR = (NROW + NTHREADS - 1) / NTHREADS;
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  const int nvalid = min(TT, A.n_traj - n0) * M::R;
  const size_t NRL = (size_t)A.n_traj * M::R * M::L;
  #pragma unroll 1
  for (int u = 0; u < PR; ++u) {
    const int i = tid + u * NTHREADS;
    if (i < nvalid) {
      const int t = i / M::R, r = i - t * M::R;
      const float* rec = lds + t * SR;
      const f4 lo = {rec[M::Y_OFF + 3 * r], rec[M::Y_OFF + 3 * r + 1], rec[M::Y_OFF + 3 * r + 2], rec[XOFF + 5 * r]};
      const f4 hi = {rec[XOFF + 5 * r + 1], rec[XOFF + 5 * r + 2], rec[XOFF + 5 * r + 3], rec[XOFF + 5 * r + 4]};
      const size_t row = ((size_t)n0 * M::R + i) * M::L;
      f4* d0 = reinterpret_cast<f4*>(A.latent + row);
      d0[0] = lo;
      d0[1] = hi;
      #pragma unroll 1
      for (int o = 0; o < A.n_out; ++o) {
        float* d = A.latent + (size_t)sc.out_j[o] * NRL + row;
        d[3] = lo[3];
        *reinterpret_cast<f4*>(d + 4) = hi;
      }
    }
  }
}

__device__ __forceinline__ size_t ckpt_index(int tile, int n_steps, int step, int stage, int F, int f, int t) {
  return ((((size_t)tile * n_steps + step) * 4 + stage) * F + f) * TT + t;
}

// The stage input in the record's Y slot ([16][F] at Y_OFF) -> its checkpoint block ([F][16]): lane
// (f, q) gathers trajectories 4q .. 4q + 3 of feature f (conflict-free LDS reads: consecutive lanes,
// consecutive banks) and writes them as one 16-B store; 64 lanes cover 1 KB of the block.
template <class M, int SR>
__device__ __forceinline__ void store_ckpt_rows(float* blk, const float* lds, int tid) {
  constexpr int NQ = M::F * (TT / 4), PER = (NQ + NTHREADS - 1) / NTHREADS;
  asm volatile("" : "+v"(tid));
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int i = tid + u * NTHREADS;
    if (i < NQ) {
      const int f = i >> 2, t0 = (i & 3) * 4;
      const f4 v = {lds[t0 * SR + M::Y_OFF + f], lds[(t0 + 1) * SR + M::Y_OFF + f],
                    lds[(t0 + 2) * SR + M::Y_OFF + f], lds[(t0 + 3) * SR + M::Y_OFF + f]};
      reinterpret_cast<f4*>(blk)[i] = v;
    }
  }
}

// GST training forward: the tiles' static features ([tile][16][S16]) behind the stage checkpoints and
// stored rows (the weight-gradient GEMM's layer-0 input beside each stage's stored input).
template <class M>
__host__ __device__ __forceinline__ size_t gst_static_off(int n_tiles, int n_steps) {
  return (size_t)n_tiles * n_steps * 4 * (M::F * TT + (M::ACT_STORED ? TT * M::XST_W : 0));
}
// DEC training forward: the solve's final state y_{n_steps} ([tile][F][16]) behind the stage
// checkpoints, stored activations and (GST) static features, i.e. at ude_query's ckpt_bytes (the
// decoder backward reads every output state from there).
template <class M>
__host__ __device__ __forceinline__ size_t ckpt_final_off(int n_tiles, int n_steps) {
  return gst_static_off<M>(n_tiles, n_steps) + (M::GST ? (size_t)n_tiles * TT * M::S16 : 0);
}

// Stored activations (Model::ACT_STORED) of one tile-stage: [16][XST_W] behind the checkpoint.
template <class M>
__host__ __device__ __forceinline__ float* act_block(float* ckpt, int n_tiles, int n_steps, int tile, int step,
                                                     int stage) {
  const size_t ck = (size_t)n_tiles * n_steps * 4 * M::F * TT;
  return ckpt + ck + (((size_t)tile * n_steps + step) * 4 + stage) * TT * M::XST_W;
}
template <class M>
constexpr int act_q_per_thread() { return (TT * M::ACT_A4 / 4 + NTHREADS - 1) / NTHREADS; }
// Quad i of a tile-stage's activation rows ([16][ACT_A4] in record order, i = t * ACT_A4 / 4 + q)
// -> its quad index in the stored block ([16][XST_W], activation rows at column ACT_IN).
template <class M>
__host__ __device__ __forceinline__ int act_src_q(int i) {
  constexpr int QR = M::ACT_A4 / 4;
  if constexpr (M::XST_W == M::ACT_A4) return i;
  else return (i / QR) * (M::XST_W / 4) + M::ACT_IN / 4 + (i - (i / QR) * QR);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Fixed-order sum of one statistic's per-workgroup partials by one wave (lane-strided, then a fixed
// butterfly): the order of ude_stats_finalize_kernel / ude_sum_finalize_kernel, so both paths give the
// same bits.  The partials are read with device-coherent loads (written by other workgroups, possibly
// on other XCDs, with device-coherent stores).
__device__ __forceinline__ double wave_sum_partials(const double* part, int n, int stride, int off, int ln) {
  double s = 0.0;
  for (int gi = ln; gi < n; gi += 64)
    s += __hip_atomic_load(part + (size_t)gi * stride + off, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m, 64);
  return s;
}

// Statistics from the per-workgroup partials, by wave 0 of the last workgroup to arrive (ticket on
// A.ctl):
//   mean_c = S_c / n, std_c = sqrt((S2_c - n mean_c^2) / (n - 1)) (torch's unbiased std,
//   lib/models.py:152-156), |Fa| = sqrt(S_Fa) (lib/VAE.py:180); DEC: latent_init_loss.
// Publication without agent-scope fences: on gfx950 those write back / invalidate the whole L2 of the
// XCD (buffer_wbl2 / buffer_inv sc1), which at the end of a forward that has just written GBs of
// checkpoints cost 52 us per launch (measured).  Instead the partials go out as device-scope (sc1)
// stores, complete (s_waitcnt vmcnt(0)) before the ticket is taken, and the last workgroup reads them
// with device-scope loads: the device-coherent path, no cache maintenance.  The counter is reset for
// the next launch (stream ordered).
//
// Ordering argument (the atomics are relaxed: under the HIP/C++ memory model alone this pattern would
// be a data race, so it rests on gfx950's hardware ordering, made explicit here):
//  1. the partials are agent-scope (sc1) stores: written through to the device-coherent level, not
//     left in a non-coherent cache;
//  2. publish_fence(): s_waitcnt vmcnt(0) -- every store of the wave has been acknowledged (is visible
//     device-wide) -- plus a compiler barrier, so no memory operation is moved across it;
//  3. only then the ticket's agent-scope fetch_add (performed at the device-coherent level, after
//     step 2 in program order);
//  4. the last arrival, after its ticket came back and another compiler barrier, reads the partials
//     with agent-scope (sc1) loads, which are served from the device-coherent level.
// An acquire / release pair at agent scope would add an L2 write-back / invalidate of the XCD
// (buffer_wbl2 / buffer_inv sc1): 52 us at the end of a forward that has just written GBs.
__device__ __forceinline__ void publish_fence() {
  __builtin_amdgcn_s_waitcnt(0x0F70);              // vmcnt(0): this wave's stores are acknowledged
  __asm__ __volatile__("" ::: "memory");           // and the compiler keeps every access on its side
}

template <bool DEC>
__device__ __forceinline__ void finalize_stats_last(const KArgs& A, int ln) {
  publish_fence();
  unsigned int ticket = 0;
  if (ln == 0) ticket = __hip_atomic_fetch_add(A.ctl, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  ticket = __builtin_amdgcn_readfirstlane(ticket);
  if (ticket != gridDim.x - 1) return;
  __asm__ __volatile__("" ::: "memory");           // the partial loads stay behind the ticket
  const int ng = gridDim.x;
  double tot[5];
#pragma unroll
  for (int c = 0; c < 5; ++c) tot[c] = wave_sum_partials(A.stats_slab, ng, 5, c, ln);
  double reg = 0.0;
  if constexpr (DEC) reg = wave_sum_partials(A.reg_slab, ng, 1, 0, ln);
  if (ln < 2) {
    const double n = A.n_eval, t0 = ln == 0 ? tot[0] : tot[1], t2 = ln == 0 ? tot[2] : tot[3];
    const double m = t0 / n;
    const double var = (t2 - n * m * m) / (n - 1.0);
    if (A.o_mean) A.o_mean[ln] = (float)m;
    if (A.o_std) A.o_std[ln] = (float)sqrt(var > 0.0 ? var : 0.0);
  }
  if (ln == 2 && A.o_norm) A.o_norm[0] = (float)sqrt(tot[4]);
  if (ln == 3 && DEC) A.o_reg[0] = (float)reg;
  if (A.o_sums && ln < 5) {
    double v = tot[0];
#pragma unroll
    for (int c = 1; c < 5; ++c) v = ln == c ? tot[c] : v;
    A.o_sums[ln] = v;
  }
  if (ln == 0) *A.ctl = 0u;
}

// ============================================================================
// Forward solve
// ============================================================================
// DEC (decoder epilogue): instead of the (T, N, R, L) latent, every output time
// emits y_hat = W_dec . y[:3R] + b_dec ((T, N, R), the Decoder of lib/models.py:27-51 as
// lib/VAE.py:138 applies it) and the latent_init_loss sum over y[..., :3] (:189); the training
// forward also stores the final state for the decoder backward.  Outputs must be grid hits
// (schedule mode 1; the host checks).
// RES (deterministic weights too large for two workgroups' registers, launched when the tiles do not
// outnumber the CUs): one workgroup per CU with every forward fragment resident in VGPRs for the whole
// launch -- no phase waits on the L2 latency of its weights (the few-tile / strong-scaling shard case,
// where no second workgroup on the CU hides it).
template <class M, bool TRAIN, int W, bool SPLIT = false, bool DEC = false, bool RES = false>
__device__ void fwd_body(const KArgs& A, float* lds) {
  constexpr int SR = M::SR_F;
  constexpr int SL = M::SLOTS;
  int tid = threadIdx.x;
  const int lane = tid & 63;
  const Sched sc(A.sched, A.n_steps, A.n_out);
  const size_t NRL = (size_t)A.n_traj * M::R * M::L;
  const Rsrc rs = make_rsrc(A.pack, M::PACK_TOTAL * 4);
  const Rsrc rsd = DEC ? make_rsrc(A.dec_pack, M::DEC_PACK * 4) : rs;
  double st_b = 0, st_g = 0, st_bb = 0, st_gg = 0, st_fa = 0;
  // DEC: this thread's latent_init_loss partial lives in LDS behind the record (the large models'
  // forward is at its 256-VGPR limit: two more live registers spilled)
  double* st_reg = reinterpret_cast<double*>(lds + M::REG_LDS_F) + tid;
  if constexpr (DEC) *st_reg = 0.0;

  // BAYES at small sizes (PFB): each evaluation's weight sample lives in registers, loaded while the
  // previous evaluation's flux pass runs (its L2 latency off the layer phases; at one tile per CU
  // nothing else on the CU hides it)
  constexpr bool PFB = M::FWD_PFB;
  WRegs<M, W, false, true, RES || PFB> wr;
  if constexpr (!PFB) wr.load(rs, lane);
  Prof prof_, *pf = nullptr;
#ifdef UDE_PROFILE
  if (TRAIN && A.prof && tid == 0) {
    pf = &prof_;
    for (int i = 0; i < NPROF; ++i) prof_.acc[i] = 0;
    prof_.last = __builtin_amdgcn_s_memtime();
  }
#endif

  #pragma unroll 1
  for (int i = tid; i < TT * SR; i += NTHREADS) lds[i] = 0.f;
  lds_sync();

  for (int tile = blockIdx.x; tile < A.n_tiles; tile += gridDim.x) {
    const int n0 = tile * TT;
    // The RK4 state and the 3/8-rule combinations are carried in fp64 (the stage evaluations stay fp32:
    // every stage input is rounded to fp32 for the MLPs, the checkpoint and the masks).  The reference's
    // torchdiffeq combination runs in fp32; on trajectories that pass next to the mask boundary of
    // lib/models.py:130 its rounding is amplified ~1e5-fold (whole-batch weight
    // gradients of the M1 FaFp batch 5x outside the fp32 oracle's spread); an fp64 state brings those
    // trajectories 2-50x closer to fp64 (tools/ns_traj.py, "fp32 rhs / fp64 state") at 3 extra VGPRs per
    // state slot and a few fp64 VALU operations per stage.
    double ys[SL][3];
    float k1[SL][3], k2[SL][3], k3[SL][3];
    // DEC: y_hat of output jo from the state in the record's Y slot (decoder row tiles over the
    // waves; no barrier: the next write of the Y slot is behind the next stage's layer barriers)
    auto dec_emit = [&](int jo) {
      if constexpr (DEC) {
        const int t = lane & 15, g = lane >> 4;
        sfor<M::RTD>([&](auto kk) {
          constexpr int k = decltype(kk)::value;
          if constexpr (k % WAVES == W) {
            f4 acc = ldw(rsd, g * 16, (M::DEC_WF + k * 16) * 4);
            acc = gemm_tile_lean<M::F16, k * (M::F16 / 16) * 256, 2>(rsd, lds + t * SR + M::Y_OFF, lane, acc);
            const int n = n0 + t;
            if (n < A.n_traj) {
              float* dst = A.yhat + ((size_t)jo * A.n_traj + n) * M::R + k * 16 + 4 * g;
#pragma unroll
              for (int e = 0; e < 4; ++e)
                if (k * 16 + 4 * g + e < M::R) dst[e] = acc[e];
            }
          }
        });
      }
    };

    // the row-mapped tile start (fwd_tile_static / fwd_tile_latent; L = 8: 16-B latent rows, checked by
    // the host entry)
    constexpr bool rows16 = M::L == 8;
    // large records: each stage's checkpointed input written as 16-B rows from the Y slot behind phase 0's
    // weight loads (state49 fwd 0.945 -> 0.925 ms); small records keep three 4-B stores per (trajectory,
    // region) in the flux pass (rows cost M1 2%; profiles/r04/ab_ck_*.log)
    constexpr bool CKR = SL > 1;
    if constexpr (rows16) fwd_tile_static<M, SR, M::XSF_OFF>(A, lds, n0);
    // y0 -> registers, LDS Y slot, latent[0], ckpt(step 0, stage 0)
    sfor<SL>([&](auto ss) {
      constexpr int sl = decltype(ss)::value;
      const int p = tid + sl * NTHREADS;
      if (p < M::PAIRS) {
        const int r = p / TT, t = p - r * TT;
        const int n = n0 + t;
        const bool valid = n < A.n_traj;
        const float* src = A.y0 + ((size_t)n * M::R + r) * M::L;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const float y = valid ? src[c] : 0.f;
          ys[sl][c] = (double)y;
          lds[t * SR + M::Y_OFF + 3 * r + c] = y;
          if (TRAIN && !CKR && A.n_steps > 0) A.ckpt[ckpt_index(tile, A.n_steps, 0, 0, M::F, 3 * r + c, t)] = y;
          if (DEC && valid) *st_reg += (double)reg_term(y);
        }
        if (valid && !DEC && !rows16) {
          float* dst = A.latent + ((size_t)n * M::R + r) * M::L;
          for (int c = 0; c < M::L; ++c) dst[c] = src[c];
        }
      }
    });
    // static latent dims (zero derivative, carried unchanged: lib/models.py:144) of every output
    // time, once per tile (not in the step loop, where each copy waited on a global load)
    if constexpr (M::L > 3 && !DEC && !rows16) {
      #pragma unroll 1
      for (int i = tid; i < A.n_out * M::PAIRS; i += NTHREADS) {
        const int o = i / M::PAIRS, p = i - o * M::PAIRS;
        const int r = p / TT, t = p - r * TT, n = n0 + t;
        if (n < A.n_traj) {
          const float* src = A.y0 + ((size_t)n * M::R + r) * M::L;
          float* dst = A.latent + (size_t)sc.out_j[o] * NRL + ((size_t)n * M::R + r) * M::L;
#pragma unroll
          for (int c = 3; c < M::L; ++c) dst[c] = src[c];
        }
      }
    }
    if constexpr (!rows16) load_static<M, SR, M::XSF_OFF>(A.y0, lds, n0, A.n_traj);
    lds_sync();
    if constexpr (TRAIN && M::GST) {
      // the tile's static features once ([tile][16][S16] behind the stored rows): the weight-gradient
      // GEMM's layer-0 input beside each stage's stored input
      f4* dst = reinterpret_cast<f4*>(A.ckpt + gst_static_off<M>(A.n_tiles, A.n_steps) + (size_t)tile * TT * M::S16);
      constexpr int QS = M::S16 / 4;
      #pragma unroll 1
      for (int i = tid; i < TT * QS; i += NTHREADS) {
        const int t = i / QS, q = i - t * QS;
        dst[i] = *reinterpret_cast<const f4*>(lds + t * SR + M::XSF_OFF + 4 * q);
      }
    }
    f4 c1[M::NZ(W) > 0 ? M::NZ(W) : 1];
    static_hoist<M, W, SR, M::XSF_OFF>(rs, lds, c1, lane);
    if constexpr (rows16 && !DEC) fwd_tile_latent<M, SR, M::XSF_OFF>(A, sc, lds, n0);
    lds_sync();                                   // the static features (aliased by the activations) are dead
    if constexpr (DEC) dec_emit(0);               // output 0 = y0
    UDE_STAMP(pf, 15);

    for (int step = 0; step < A.n_steps; ++step) {
      // DEC (R=49, at the 256-VGPR limit): the thread-derived 64-bit store addresses are recomputed
      // each step rather than hoisted out of the loop and spilled (each reload waited on every
      // checkpoint / activation store in flight)
      if constexpr (DEC) asm volatile("" : "+v"(tid));
      const float dt = sc.dt[step];
      for (int j = 0; j < 4; ++j) {
        // BAYES: evaluation 4 step + j has its own weight sample
        Rsrc rse = rs;
        if constexpr (M::BAYES) rse = make_rsrc(A.pack + (size_t)(4 * step + j) * M::PACK_TOTAL, M::PACK_TOTAL * 4);
        if constexpr (PFB) {
          if (step == 0 && j == 0) wr.load(rse, lane, false);        // the tile's first evaluation
        }
        // this stage's input (the record's Y slot, layer 0's input) -> its checkpoint, issued behind
        // phase 0's weight loads (their waits then do not wait for these stores) and read before
        // the phase's barrier (the flux pass overwrites the slot after the last phase)
        mlp_forward<M, W, SR>(rse, lds, c1, lane, wr, pf, [&](auto dd) {
          if constexpr (decltype(dd)::value == 0) {
            if constexpr (TRAIN && CKR)
              store_ckpt_rows<M, SR>(A.ckpt + ckpt_index(tile, A.n_steps, step, j, M::F, 0, 0), lds, tid);
          }
        });
        if constexpr (PFB) {
          const int en = 4 * step + j + 1;
          if (en < 4 * A.n_steps) wr.load(make_rsrc(A.pack + (size_t)en * M::PACK_TOTAL, M::PACK_TOTAL * 4), lane, false);
        }
        if constexpr (TRAIN && M::ACT_STORED && !SPLIT && UDE_ABL != 11) {
          // this stage's activation rows -> HBM for the backward (read before the flux barrier;
          // the stores drain behind the rest of the stage)
          f4* dst = reinterpret_cast<f4*>(act_block<M>(A.ckpt, A.n_tiles, A.n_steps, tile, step, j));
          constexpr int QR = M::ACT_A4 / 4, NQ = act_q_per_thread<M>();
          // all of a thread's LDS reads, then all its 16-B stores (state49 fwd 0.936 -> 0.892 ms against
          // batches of 3 quads, profiles/r04/ab_uc_*.log: the phases' registers are free by then)
          constexpr int UC = NQ <= 5 ? NQ : cmin(NQ, 16);
          #pragma unroll 1
          for (int u0 = 0; u0 < NQ; u0 += UC) {
#pragma unroll
            for (int uu = 0; uu < UC; ++uu) {
              const int i = tid + (u0 + uu) * NTHREADS;
              if (u0 + uu < NQ && i < TT * QR) {
                const int t = i / QR, q = i - t * QR;
                dst[act_src_q<M>(i)] = *reinterpret_cast<const f4*>(lds + t * SR + M::ACT0 + 4 * q);
              }
            }
          }
        }
        UDE_STAMP(pf, 0);
        if constexpr (UDE_ABL != 12) sfor<SL>([&](auto ss) {
          constexpr int sl = decltype(ss)::value;
          const int p = tid + sl * NTHREADS;
          if (p < M::PAIRS) {
            const int r = p / TT, t = p - r * TT;
            const int n = n0 + t;
            const bool valid = n < A.n_traj;
            float* rec = lds + t * SR;
            float Y[3], f[3];
#pragma unroll
            for (int c = 0; c < 3; ++c) Y[c] = rec[M::Y_OFF + 3 * r + c];
            if constexpr (TRAIN && M::GST) {
              // the stage input in front of the stored activation rows (the layer-0 input of the
              // weight-gradient GEMM); its pad columns [F, F16) zeroed by the last region's threads
              float* xrow = act_block<M>(A.ckpt, A.n_tiles, A.n_steps, tile, step, j) + t * M::XST_W;
#pragma unroll
              for (int c = 0; c < 3; ++c) xrow[3 * r + c] = Y[c];
              if (r == M::R - 1)
                for (int c = M::F; c < M::F16; ++c) xrow[c] = 0.f;
            }
            if constexpr (M::HAS_P) {
              const float q0 = rec[M::act_off(0, M::nl(0) - 1) + 2 * r];
              const float q1 = rec[M::act_off(0, M::nl(0) - 1) + 2 * r + 1];
              const float b = fabsf(q0), gm = fabsf(q1);
              const float plus = (b * Y[0]) * Y[1];
              const float minus = gm * Y[1];
              f[0] = -plus; f[1] = plus - minus; f[2] = minus;
              if (valid && UDE_ABL != 14) {
                st_b += (double)b; st_g += (double)gm;
                st_bb += (double)b * (double)b; st_gg += (double)gm * (double)gm;
              }
            }
            if constexpr (M::HAS_A) {
#pragma unroll
              for (int c = 0; c < 3; ++c) {
                const float fa = rec[M::act_off(1, M::nl(1) - 1) + 3 * r + c];
                if constexpr (M::HAS_P) f[c] = f[c] + A.fa_w * fa;
                else f[c] = fa;
                if (valid && UDE_ABL != 14) st_fa += (double)fa * (double)fa;
              }
            }
#pragma unroll
            for (int c = 0; c < 3; ++c) f[c] = (Y[c] > 2.f || Y[c] < -1.f) ? 0.f : f[c];
            float Yn[3];
            const double dd = (double)dt;
            if (j == 0) {
#pragma unroll
              for (int c = 0; c < 3; ++c) {
                k1[sl][c] = f[c];
                Yn[c] = (float)(ys[sl][c] + (dd * (double)f[c]) * (1.0 / 3.0));
              }
            } else if (j == 1) {
#pragma unroll
              for (int c = 0; c < 3; ++c) {
                k2[sl][c] = f[c];
                Yn[c] = (float)(ys[sl][c] + dd * ((double)f[c] - (double)k1[sl][c] * (1.0 / 3.0)));
              }
            } else if (j == 2) {
#pragma unroll
              for (int c = 0; c < 3; ++c) {
                k3[sl][c] = f[c];
                Yn[c] = (float)(ys[sl][c] + dd * (((double)k1[sl][c] - (double)k2[sl][c]) + (double)f[c]));
              }
            } else {
              float yold[3];
#pragma unroll
              for (int c = 0; c < 3; ++c) {
                yold[c] = (float)ys[sl][c];
                const double dy =
                    ((((double)k1[sl][c] + 3.0 * ((double)k2[sl][c] + (double)k3[sl][c])) + (double)f[c]) * dd) * 0.125;
                ys[sl][c] = ys[sl][c] + dy;
                Yn[c] = (float)ys[sl][c];
              }
              if constexpr (DEC) {
                // every output is a grid hit (mode 1): latent_init_loss of the new state; y_hat
                // follows from the record after the barrier (dec_emit)
                if (valid && sc.out_start[step] < sc.out_start[step + 1]) {
#pragma unroll
                  for (int c = 0; c < 3; ++c) *st_reg += (double)reg_term(Yn[c]);
                }
                if (TRAIN && step == A.n_steps - 1) {
#pragma unroll
                  for (int c = 0; c < 3; ++c) A.ckpt_final[((size_t)tile * M::F + 3 * r + c) * TT + t] = Yn[c];
                }
              } else if (valid && UDE_ABL != 16) {
                const int o_end = sc.out_start[step + 1];
                #pragma unroll 1
                for (int o = sc.out_start[step]; o < o_end; ++o) {
                  const int jo = sc.out_j[o], mode = sc.out_mode[o];
                  const float slope = sc.out_slope[o];
                  float* dst = A.latent + (size_t)jo * NRL + ((size_t)n * M::R + r) * M::L;
                  float v[3];
#pragma unroll
                  for (int c = 0; c < 3; ++c) {
                    if (mode == 0) v[c] = yold[c];
                    else if (mode == 1) v[c] = Yn[c];
                    else v[c] = yold[c] + slope * (Yn[c] - yold[c]);
                  }
                  if constexpr (rows16) {
                    // 16-B aligned 32-B rows (host entry check): one 12-byte store per (trajectory,
                    // region) instead of three (the stores' issue was 4.6% of the state49 forward)
                    __builtin_memcpy(__builtin_assume_aligned(dst, 16), v, 12);
                  } else {
#pragma unroll
                    for (int c = 0; c < 3; ++c) dst[c] = v[c];
                  }
                }
              }
            }
#pragma unroll
            for (int c = 0; c < 3; ++c) rec[M::Y_OFF + 3 * r + c] = Yn[c];
            if (TRAIN) {
              const int ns = j == 3 ? step + 1 : step;
              const int nj = j == 3 ? 0 : j + 1;
              if (!CKR && ns < A.n_steps && UDE_ABL != 15) {
#pragma unroll
                for (int c = 0; c < 3; ++c)
                  A.ckpt[ckpt_index(tile, A.n_steps, ns, nj, M::F, 3 * r + c, t)] = Yn[c];
              }
            }
          }
        });
        UDE_STAMP(pf, 16);
        lds_sync();
        UDE_STAMP(pf, 1);
      }
      if constexpr (DEC) {
        if (sc.out_start[step] < sc.out_start[step + 1]) dec_emit(sc.out_j[sc.out_start[step]]);
      }
    }
  }

  // deterministic per-workgroup partial sums
  constexpr int NS = DEC ? 6 : 5;
  double* red = reinterpret_cast<double*>(lds);
  double v[6] = {wave_sum(st_b), wave_sum(st_g), wave_sum(st_bb), wave_sum(st_gg), wave_sum(st_fa),
                 DEC ? wave_sum(*st_reg) : 0.0};
  lds_sync();
  if (lane == 0) {
#pragma unroll
    for (int c = 0; c < NS; ++c) red[(tid >> 6) * NS + c] = v[c];
  }
  lds_sync();
  if (tid < NS) {
    double s = 0;
    for (int w = 0; w < WAVES; ++w) s += red[w * NS + tid];
    double* dst = tid < 5 ? A.stats_slab + (size_t)blockIdx.x * 5 + tid : A.reg_slab + blockIdx.x;
    // in-kernel finalize (ctl): device-coherent store, read back by the last workgroup (see
    // finalize_stats_last)
    if (A.ctl) __hip_atomic_store(dst, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *dst = s;
  }
  // the last workgroup to finish turns every workgroup's partials into the statistics (no separate
  // finalize launch; wave 0 only, so the split forward's partner waves keep their barrier sequence)
  if (A.ctl && tid < 64) finalize_stats_last<DEC>(A, tid);
#ifdef UDE_PROFILE
  if (pf) for (int i = 0; i < NPROF; ++i) A.prof[(size_t)blockIdx.x * NPROF + i] = prof_.acc[i];
#endif
}

// Training forward of small records (Model::split_fwd): waves 4-7 store each stage's activation
// rows (the backward's input) from the record to HBM while waves 0-3 run the flux pass; the same
// barrier sequence as fwd_body.
template <class M, bool DEC>
__device__ void fwd_sbody(const KArgs& A, float* lds) {
  constexpr int SR = M::SR_F;
  constexpr int QR = M::ACT_A4 / 4, NQ = act_q_per_thread<M>();
  const int wt = threadIdx.x - NTHREADS;
  lds_sync();                                  // record zeroed
  for (int tile = blockIdx.x; tile < A.n_tiles; tile += gridDim.x) {
    lds_sync();                                // tile inputs in the record
    lds_sync();                                // static hoist
    for (int step = 0; step < A.n_steps; ++step) {
      #pragma unroll 1
      for (int j = 0; j < 4; ++j) {
        sfor<M::D>([&](auto) { lds_sync(); }); // the MLP phases
        f4* dst = reinterpret_cast<f4*>(act_block<M>(A.ckpt, A.n_tiles, A.n_steps, tile, step, j));
        f4 v[NQ];
#pragma unroll
        for (int u = 0; u < NQ; ++u) {
          const int i = wt + u * NTHREADS;
          if (i < TT * QR) {
            const int t = i / QR, q = i - t * QR;
            v[u] = *reinterpret_cast<const f4*>(lds + t * SR + M::ACT0 + 4 * q);
          }
        }
#pragma unroll
        for (int u = 0; u < NQ; ++u) {
          const int i = wt + u * NTHREADS;
          if (i < TT * QR) dst[act_src_q<M>(i)] = v[u];
        }
        lds_sync();                            // flux pass (the next stage rewrites the rows)
      }
    }
  }
  lds_sync();                                  // side-statistic reduction
  lds_sync();
}

// SPLIT (training, Model::split_fwd, launched when every tile has a CU of its own): 8 waves.
// DEC: the decoder epilogue (y_hat and latent_init_loss, no latent).
template <class M, bool TRAIN, bool SPLIT = false, bool DEC = false, bool RES = false>
__global__ __launch_bounds__(SPLIT ? 2 * NTHREADS : NTHREADS, (SPLIT || RES) ? 1 : 2) void ude_fwd_kernel(KArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if constexpr (SPLIT) {
    if (w >= WAVES) { fwd_sbody<M, DEC>(a, lds); return; }
  }
  if (w == 0) fwd_body<M, TRAIN, 0, SPLIT, DEC, RES>(a, lds);
  else if (w == 1) fwd_body<M, TRAIN, 1, SPLIT, DEC, RES>(a, lds);
  else if (w == 2) fwd_body<M, TRAIN, 2, SPLIT, DEC, RES>(a, lds);
  else fwd_body<M, TRAIN, 3, SPLIT, DEC, RES>(a, lds);
}

// ============================================================================
// Backward (VJP)
// ============================================================================
// RK4 (3/8 rule) adjoint of the stage input, MLP part: consumes the layer-0 input
// gradient dY (4 features x 1 trajectory per lane) straight from the dX tile's
// registers (see the flux section of bwd_body for the direct part).
template <class M, int SR>
struct RkAdjointEp {
  float* rec;      // this lane's trajectory record
  float dt;
  int jj;          // RK stage (3..0)
  __device__ __forceinline__ void operator()(int f0, f4 dY) const {
    if constexpr (M::FULL0) {
      // static features (rows F16..): no RK adjoint, their input gradient is summed
      // over every evaluation of the solve (DYS, written to dy0 at tile end)
      if (f0 >= M::F16) {
        *reinterpret_cast<f4*>(rec + M::DYS_OFF + f0 - M::F16) += dY;
        return;
      }
    }
    if (f0 >= M::F4) return;                       // padded feature rows
    // DYF: the stage's flux part (parked by the flux pass) joins the MLP part first, one update
    if constexpr (M::DYF) dY += *reinterpret_cast<const f4*>(rec + M::DYF_OFF + f0);
    f4* accy = reinterpret_cast<f4*>(rec + M::RK_ACCY + f0);
    f4* dk1 = reinterpret_cast<f4*>(rec + M::RK_DK1 + f0);
    f4* dk2 = reinterpret_cast<f4*>(rec + M::RK_DK2 + f0);
    f4* dk3 = reinterpret_cast<f4*>(rec + M::RK_DK3 + f0);
    // every read before the first write: one LDS round trip, not one per accumulator
    const f4 a = *accy, k1 = *dk1, k2 = *dk2, k3 = *dk3;
    rk_adjoint_update(dY, dt, jj, a, k1, k2, k3, accy, dk1, dk2, dk3);
  }
  // 3/8-rule stage-input adjoint: accy += dY and the stage cotangents of the stages before jj
  //   Y2 = y + (dt k1)/3, Y3 = y + dt (k2 - k1/3), Y4 = y + dt (k1 - k2 + k3)
  static __device__ __forceinline__ void rk_adjoint_update(f4 dY, float dt, int jj, f4 a, f4 k1, f4 k2, f4 k3,
                                                           f4* accy, f4* dk1, f4* dk2, f4* dk3) {
    *accy = a + dY;
    if (jj == 3) {
      const f4 u = dt * dY;
      *dk1 = k1 + u; *dk2 = k2 - u; *dk3 = k3 + u;
    } else if (jj == 2) {
      const f4 u = dt * dY;
      *dk2 = k2 + u; *dk1 = k1 - u * (1.0f / 3.0f);
    } else if (jj == 1) {
      *dk1 = k1 + (dY * (1.0f / 3.0f)) * dt;
    }
  }
};

// BAYES: `es` addresses this evaluation's eps in slab order; every tile's dW
// contribution of the evaluation is also accumulated eps-weighted into `dws` (and the
// bias row sums into DBS): d|std| = sum_eval eps_eval * dW_eval (models_bayes.py:45-46).
// DX_ONLY (SPLIT_BWD critical-path waves): only the input gradients; the weight gradients of
// the phase are the partner waves' (mlp_backward_dw).
// GST: the wave's owned rows of every layer-output gradient also go to `gblk` (this tile-stage's
// [16][ACT_A4] block, record column order) for ude_gst_dw_kernel.
// GST (no weight-gradient work, registers to spare): the input-gradient fragments come from `fxp`
// ([WX_Q(W)] quads, phase d at xq_base(W, d)), each phase's loaded while the previous phase runs
// (the caller issues the first phase's before the flux pass), so no phase waits on the L2 latency.
template <class M, int W, int SR, bool DX_ONLY = false, bool PFX = false, class DW, class DS, class G0, class EP0,
          class WR>
__device__ __forceinline__ void mlp_backward(Rsrc rs, Rsrc es, float* lds, DW& dw, DS& dws, G0& g0t, int lane,
                                             Prof* pf, const EP0& ep0, const WR& wr, float* gblk = nullptr,
                                             f4* fxp = nullptr) {
  constexpr bool RW = WR::ON;
  constexpr bool PF = PFX && !RW;     // only the RK4 backward (bwd_body) hands over the fxp array
  const int t = lane & 15, g = lane >> 4;
  float* rec = lds + t * SR;
  sfor<M::D>([&](auto ee) {
    constexpr int d = M::D - 1 - decltype(ee)::value;
    UDE_STAMP(pf, 24 + d);
    // input-gradient fragments go out first; the LDS-only dW GEMMs below hide them
    constexpr int NX = M::XQ(W, d);
    f4 fx[(NX > 0 && !RW && !PF) ? NX : 1];
    if constexpr (!RW && !PF) load_x_frags<M, W, d>(rs, lane, fx);
    auto FX = [&](int i) -> f4 {
      if constexpr (RW) return wr.wx[M::xq_base(W, d) + i];
      else if constexpr (PF) return fxp[M::xq_base(W, d) + i];
      else return fx[i];
    };
    // BAYES: this evaluation's eps for the wave's dW tiles (C layout) and bias rows
    constexpr int NE = (M::BAYES && !DX_ONLY) ? M::ndw_phase(W, d) : 0;
    f4 ef[NE > 0 ? NE : 1], eb[M::FT(d) > 0 ? M::FT(d) : 1];
    if constexpr (M::BAYES && !DX_ONLY) {
      sfor<M::FT(d)>([&](auto kk) {
        constexpr int k = decltype(kk)::value;
        if constexpr (M::fowner(d, k) == W) {
          constexpr int e0 = M::ndw_before(W, d, k) - M::ndw_before(W, d, 0);
          sfor<M::rti(M::fnet(d, k), d)>([&](auto cc) {
            constexpr int ct = decltype(cc)::value;
            ef[e0 + ct] = ldw(es, lane * 16, (M::dyn_tiles_before(d, k) + ct) * 1024);
          });
          eb[k] = ldw(es, g * 16, (M::SLAB_DB + (M::FTbase(d) + k) * 16) * 4);
        }
      });
    }
    __builtin_amdgcn_sched_barrier(0);
    // (1) rows owned by this wave: bias/G sums and the dW GEMM (K = trajectories).
    // When they fit, every owned tile's LDS operands are read before the first MFMA
    // (one LDS latency per phase instead of one per tile).
    constexpr int NOWN = M::own_phase(W, d);
    constexpr int NDP = M::ndw_phase(W, d);
    constexpr bool BATCH = !DX_ONLY && !M::BAYES && NOWN > 0 && 4 * NOWN * 2 + 4 * NDP <= 96;
    if constexpr (BATCH) {
      f4 gvv[NOWN];
      float gaa[NOWN][4], bva[NDP][4];
      sfor<M::FT(d)>([&](auto kk) {
        constexpr int k = decltype(kk)::value;
        if constexpr (M::fowner(d, k) == W) {
          constexpr int net = M::fnet(d, k), rt = M::frt(d, k), goff = M::gbuf(net, d);
          constexpr int inoff = d == 0 ? M::Y_OFF : M::act_off(net, d - 1);
          constexpr int o = M::ng_before(W, d, k) - M::ng_before(W, d, 0);
          constexpr int e0 = M::ndw_before(W, d, k) - M::ndw_before(W, d, 0);
          gvv[o] = *reinterpret_cast<const f4*>(rec + goff + rt * 16 + g * 4);
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            gaa[o][s] = lds[(4 * g + s) * SR + goff + rt * 16 + t];
            sfor<M::rti(net, d)>([&](auto cc) {
              constexpr int ct = decltype(cc)::value;
              bva[e0 + ct][s] = lds[(4 * g + s) * SR + inoff + ct * 16 + t];
            });
          }
        }
      });
      __builtin_amdgcn_sched_barrier(0);
      sfor<M::FT(d)>([&](auto kk) {
        constexpr int k = decltype(kk)::value;
        if constexpr (M::fowner(d, k) == W) {
          constexpr int net = M::fnet(d, k);
          constexpr int o = M::ng_before(W, d, k) - M::ng_before(W, d, 0);
          constexpr int e0 = M::ndw_before(W, d, k) - M::ndw_before(W, d, 0);
#pragma unroll
          for (int s = 0; s < 4; ++s)
            sfor<M::rti(net, d)>([&](auto cc) {
              constexpr int ct = decltype(cc)::value;
              constexpr int idx = M::ndw_before(W, d, k) + ct;
              dw[idx] = mfma4(gaa[o][s], bva[e0 + ct][s], dw[idx]);
            });
          if constexpr (d == 0) {
            g0t[M::nz_before(W, k)] += gvv[o];
          } else {
            f4 r = gvv[o];
#pragma unroll
            for (int e = 0; e < 4; ++e) r[e] = row16_sum(r[e]);
            if (t == 0) {
              float* db = lds + M::DB_LDS + (M::FTbase(d) + k) * 16 + g * 4;
              db[0] += r[0]; db[1] += r[1]; db[2] += r[2]; db[3] += r[3];
            }
          }
        }
      });
      __builtin_amdgcn_sched_barrier(0);
    } else if constexpr (!DX_ONLY)
    sfor<M::FT(d)>([&](auto kk) {
      constexpr int k = decltype(kk)::value;
      if constexpr (M::fowner(d, k) == W) {
        constexpr int net = M::fnet(d, k);
        constexpr int rt = M::frt(d, k);
        constexpr int goff = M::gbuf(net, d);
        constexpr int inoff = d == 0 ? M::Y_OFF : M::act_off(net, d - 1);
        const f4 gv = *reinterpret_cast<const f4*>(rec + goff + rt * 16 + g * 4);
        if constexpr (d == 0 && !M::BAYES) {
          g0t[M::nz_before(W, k)] += gv;          // per-trajectory sums: static-feature gradients
        } else {
          // bias gradient: sum over the tile's 16 trajectories, then into this
          // wave's rows of the workgroup's LDS row sums (fixed order: deterministic)
          f4 r = gv;
#pragma unroll
          for (int e = 0; e < 4; ++e) r[e] = row16_sum(r[e]);
          if (t == 0) {
            float* db = lds + M::DB_LDS + (M::FTbase(d) + k) * 16 + g * 4;
            db[0] += r[0]; db[1] += r[1]; db[2] += r[2]; db[3] += r[3];
            if constexpr (M::BAYES) {
              float* dbs = lds + M::DBS_LDS + (M::FTbase(d) + k) * 16 + g * 4;
              const f4 e = eb[k];
              dbs[0] += r[0] * e[0]; dbs[1] += r[1] * e[1]; dbs[2] += r[2] * e[2]; dbs[3] += r[3] * e[3];
            }
          }
        }
        // all of the tile's LDS operands are read before its first MFMA: one LDS
        // latency per tile instead of one per MFMA pair
        constexpr int NC = M::rti(net, d);
        float ga[4], bv[4][NC];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          ga[s] = lds[(4 * g + s) * SR + goff + rt * 16 + t];
#pragma unroll
          for (int ct = 0; ct < NC; ++ct) bv[s][ct] = lds[(4 * g + s) * SR + inoff + ct * 16 + t];
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (M::BAYES) {
          // this evaluation's tile contribution on its own, then into both sums
          f4 tmp[NC];
          sfor<NC>([&](auto cc) { tmp[decltype(cc)::value] = f4zero(); });
#pragma unroll
          for (int s = 0; s < 4; ++s)
            sfor<NC>([&](auto cc) {
              constexpr int ct = decltype(cc)::value;
              tmp[ct] = mfma4(ga[s], bv[s][ct], tmp[ct]);
            });
          sfor<NC>([&](auto cc) {
            constexpr int ct = decltype(cc)::value;
            constexpr int idx = M::ndw_before(W, d, k) + ct;
            constexpr int e0 = M::ndw_before(W, d, k) - M::ndw_before(W, d, 0);
            dw[idx] += tmp[ct];
            dws[idx] += tmp[ct] * ef[e0 + ct];
          });
        } else {
          // s outer: consecutive MFMAs update different dW tiles (no accumulator chain)
#pragma unroll
          for (int s = 0; s < 4; ++s)
            sfor<NC>([&](auto cc) {
              constexpr int ct = decltype(cc)::value;
              constexpr int idx = M::ndw_before(W, d, k) + ct;
              dw[idx] = mfma4(ga[s], bv[s][ct], dw[idx]);
            });
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    });
    if constexpr (M::GST) {
      sfor<M::FT(d)>([&](auto kk) {
        constexpr int k = decltype(kk)::value;
        if constexpr (M::fowner(d, k) == W) {
          constexpr int net = M::fnet(d, k), rt = M::frt(d, k);
          const f4 gv = *reinterpret_cast<const f4*>(rec + M::gbuf(net, d) + rt * 16 + g * 4);
          *reinterpret_cast<f4*>(gblk + t * M::ACT_A4 + (M::act_off(net, d) - M::ACT0) + rt * 16 + g * 4) = gv;
        }
      });
    }
    // (2) gradient w.r.t. the layer input (rows = input features); tiles sharing a
    // B operand (the same net's output gradient) are interleaved
    f4 xa[M::XT(d) > 0 ? M::XT(d) : 1];
    if constexpr (d == 0 && M::SPLITX0) {
      // partial input gradient of every layer-0 tile over this wave's K quads, to LDS;
      // summed (fixed wave order) and fed to the RK adjoint by bwd_body after the barrier
      constexpr int PQ = M::HAS_P ? M::kout(0, 0) / 16 : 0;
      // two accumulation chains per tile (even / odd K steps): half the dependent-MFMA latency
      f4 xo[M::XT(0)];
      sfor<M::XT(0)>([&](auto mm) { xa[decltype(mm)::value] = f4zero(); xo[decltype(mm)::value] = f4zero(); });
      f4 xq[M::x0q_w(W) > 0 ? M::x0q_w(W) : 1];
      sfor<M::x0q_w(W)>([&](auto jj) {
        constexpr int j = decltype(jj)::value, qq = W + j * WAVES;
        constexpr int net = qq < PQ ? 0 : 1, q = qq < PQ ? qq : qq - PQ;
        constexpr int KP = M::kout(net, 0);
        xq[j] = *reinterpret_cast<const f4*>(rec + M::gbuf(net, 0) + g * (KP / 4) + 4 * q);
      });
      sfor<M::x0q_w(W)>([&](auto jj) {
        constexpr int j = decltype(jj)::value;
        const f4 x = xq[j];
#pragma unroll
        for (int e = 0; e < 4; e += 2)
          sfor<M::XT(0)>([&](auto mm) {
            constexpr int m = decltype(mm)::value;
            xa[m] = mfma4(FX(m * M::x0q_w(W) + j)[e], x[e], xa[m]);
            xo[m] = mfma4(FX(m * M::x0q_w(W) + j)[e + 1], x[e + 1], xo[m]);
          });
      });
      sfor<M::XT(0)>([&](auto mm) {
        constexpr int m = decltype(mm)::value;
        *reinterpret_cast<f4*>(lds + M::X0P_LDS + ((W * M::XT(0) + m) * 64 + lane) * 4) = xa[m] + xo[m];
      });
      lds_sync();
      UDE_STAMP(pf, 7 + d);
      return;
    }
    f4 avv[M::XT(d) > 0 ? M::XT(d) : 1];
    sfor<M::XT(d)>([&](auto mm) {
      constexpr int m = decltype(mm)::value;
      if constexpr (M::xowner(d, m) == W) {
        xa[m] = f4zero();
        if constexpr (d > 0) {
          // the ELU-derivative operand of the epilogue, read ahead of the MFMAs
          constexpr int net = M::xnet(d, m), rt = M::xrt(d, m);
          if constexpr (M::act(net, d - 1))
            avv[m] = *reinterpret_cast<const f4*>(rec + M::act_off(net, d - 1) + rt * 16 + g * 4);
        }
      }
    });
    sfor<2>([&](auto nn) {
      constexpr int net = decltype(nn)::value;
      if constexpr (RW && packo<M>(net, d) && M::owns_x(W, d, net)) {
        // packo: one MFMA per tile, lane (t, g) supplies output g's gradient (padded rows are zero)
        const float xg = rec[M::gbuf(net, d) + g];
        sfor<M::XT(d)>([&](auto mm) {
          constexpr int m = decltype(mm)::value;
          if constexpr (M::xowner(d, m) == W && M::xnet(d, m) == net)
            xa[m] = mfma4(wr.wo[WR::po_index(d, m)], xg, xa[m]);
        });
      } else if constexpr (M::has(net, d) && M::owns_x(W, d, net)) {
        constexpr int KP = M::kout(net, d);
        // d == 0: both nets' fragments of a tile sit back to back (P first)
        constexpr int qoff = (d == 0 && net == 1 && M::HAS_P) ? M::kout(0, 0) / 16 : 0;
        const float* b = rec + M::gbuf(net, d) + g * (KP / 4);
        f4 xb[KP / 16];
#pragma unroll
        for (int q = 0; q < KP / 16; ++q) xb[q] = *reinterpret_cast<const f4*>(b + 4 * q);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < KP / 16; ++q) {
          const f4 x = xb[q];
#pragma unroll
          for (int e = 0; e < 4; ++e)
            sfor<M::XT(d)>([&](auto mm) {
              constexpr int m = decltype(mm)::value;
              if constexpr (M::xowner(d, m) == W && (d == 0 || M::xnet(d, m) == net)) {
                if constexpr (UDE_ABL == 3) xa[m][e] += x[e];
                else xa[m] = mfma4(FX(M::xq_before(W, d, m) + qoff + q)[e], x[e], xa[m]);
              }
            });
        }
      }
    });
    if constexpr (PF && d > 0) load_x_frags<M, W, d - 1>(rs, lane, fxp + M::xq_base(W, d - 1));
    sfor<M::XT(d)>([&](auto mm) {
      constexpr int m = decltype(mm)::value;
      if constexpr (M::xowner(d, m) == W) {
        f4 acc = xa[m];
        if constexpr (d == 0) {
          ep0(m * 16 + g * 4, acc);
        } else {
          constexpr int net = M::xnet(d, m);
          constexpr int rt = M::xrt(d, m);
          if constexpr (M::act(net, d - 1)) {
            const f4 av = avv[m];
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[e] = av[e] <= 0.f ? acc[e] * (av[e] + 1.f) : acc[e];
          }
          *reinterpret_cast<f4*>(rec + M::gbuf(net, d - 1) + rt * 16 + g * 4) = acc;
        }
      }
    });
    UDE_STAMP(pf, 20 + d);
    lds_sync();
    UDE_STAMP(pf, 7 + d);
  });
}

// Weight gradients of one backward stage on the SPLIT_BWD partner waves (W = the index of the
// critical-path wave sharing the SIMD): the same barrier sequence as mlp_backward, and in phase
// d the rows the wave owns: dW += g . in^T (MFMA, K = the tile's 16 trajectories) from the
// phase's LDS operands, and per-trajectory bias sums in registers (reduced over the trajectories
// once, at the launch end, instead of a cross-lane reduction every phase).
template <class M, int W, int SR>
__device__ __forceinline__ void mlp_backward_dw(const float* lds, f4* dw, f4* g0t, f4* gacc, int lane) {
  const int t = lane & 15, g = lane >> 4;
  const float* rec = lds + t * SR;
  sfor<M::D>([&](auto ee) {
    constexpr int d = M::D - 1 - decltype(ee)::value;
    sfor<M::FT(d)>([&](auto kk) {
      constexpr int k = decltype(kk)::value;
      if constexpr (M::fowner(d, k) == W && !(UDE_ABL == 6 && d == 1)) {
        constexpr int net = M::fnet(d, k), rt = M::frt(d, k), goff = M::gbuf(net, d);
        constexpr int inoff = d == 0 ? M::Y_OFF : M::act_off(net, d - 1);
        constexpr int NC = M::rti(net, d);
        const f4 gv = *reinterpret_cast<const f4*>(rec + goff + rt * 16 + g * 4);
        float ga[4], bv[4][NC];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          ga[s] = lds[(4 * g + s) * SR + goff + rt * 16 + t];
#pragma unroll
          for (int ct = 0; ct < NC; ++ct) bv[s][ct] = lds[(4 * g + s) * SR + inoff + ct * 16 + t];
        }
        if constexpr (d == 0) g0t[M::nz_before(W, k)] += gv;
        else gacc[M::ng_before(W, d, k)] += gv;
#pragma unroll
        for (int s = 0; s < 4; ++s)
          sfor<NC>([&](auto cc) {
            constexpr int ct = decltype(cc)::value;
            constexpr int idx = M::ndw_before(W, d, k) + ct;
            dw[idx] = mfma4(ga[s], bv[s][ct], dw[idx]);
          });
      }
    });
    lds_sync();
  });
}

// Cotangents of the outputs written after RK step `step` (torchdiffeq's
// _linear_interp between y_step and y_step+1): sg = the y_{step+1}-side share,
// pg = the y_step-side share, per pair slot (p = tid + sl * NTHREADS) and S/I/R.
// out_issue starts the loads of the step's first output (if any); out_finish turns
// them into shares and handles any further outputs of the step synchronously.
template <class M>
__device__ __forceinline__ void out_load(const KArgs& A, const Sched& sc, int o, int n0,
                                         float (&gv)[M::SLOTS][3], int tid = threadIdx.x) {
  // one source: the full (T, N, R, L) cotangent, or the compact S, I, R one (exactly one of
  // them is set, see ude_rk4_backward_sir)
  const int ld = A.dlatent ? M::L : 3;
  const float* gl = (A.dlatent ? A.dlatent : A.dlat_sir) + (size_t)sc.out_j[o] * A.n_traj * M::R * ld;
  sfor<M::SLOTS>([&](auto ss) {
    constexpr int sl = decltype(ss)::value;
    const int p = tid + sl * NTHREADS;
    const int r = p / TT, t = p - r * TT, n = n0 + t;
    const bool valid = p < M::PAIRS && n < A.n_traj;
    const size_t base = valid ? ((size_t)n * M::R + r) * ld : 0;
#pragma unroll
    for (int c = 0; c < 3; ++c) gv[sl][c] = valid ? gl[base + c] : 0.f;
  });
}
template <class M>
__device__ __forceinline__ void out_issue(const KArgs& A, const Sched& sc, int step, int n0,
                                          float (&gv)[M::SLOTS][3], int tid = threadIdx.x) {
  if (sc.out_start[step] < sc.out_start[step + 1]) out_load<M>(A, sc, sc.out_start[step], n0, gv, tid);
}
template <class M>
__device__ __forceinline__ void out_finish(const KArgs& A, const Sched& sc, int step, int n0,
                                           float (&gv)[M::SLOTS][3], float (&sg)[M::SLOTS][3],
                                           float (&pg)[M::SLOTS][3], int tid = threadIdx.x) {
#pragma unroll
  for (int sl = 0; sl < M::SLOTS; ++sl)
#pragma unroll
    for (int c = 0; c < 3; ++c) { sg[sl][c] = 0.f; pg[sl][c] = 0.f; }
  const int o_beg = sc.out_start[step], o_end = sc.out_start[step + 1];
  #pragma unroll 1
  for (int o = o_beg; o < o_end; ++o) {
    if (o > o_beg) out_load<M>(A, sc, o, n0, gv, tid);
    const int mode = sc.out_mode[o];
    const float slope = sc.out_slope[o];
#pragma unroll
    for (int sl = 0; sl < M::SLOTS; ++sl)
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float a = mode == 2 ? slope * gv[sl][c] : (mode == 1 ? gv[sl][c] : 0.f);
        const float b = mode == 2 ? gv[sl][c] - a : (mode == 0 ? gv[sl][c] : 0.f);
        sg[sl][c] += a;
        pg[sl][c] += b;
      }
  }
}

// Issue the loads of one checkpointed stage input ([f][t] per tile-stage in HBM)
// into registers, slot sl of thread tid holding pair p = tid + sl * NTHREADS.
template <class M>
__device__ __forceinline__ void ckpt_issue(const KArgs& A, int tile, int step, int jj, float (&ck)[M::SLOTS][3],
                                           int tid = threadIdx.x) {
  const Rsrc rck = make_rsrc(A.ckpt + ckpt_index(tile, A.n_steps, step, jj, M::F, 0, 0), M::F * TT * 4);
  sfor<M::SLOTS>([&](auto ss) {
    constexpr int sl = decltype(ss)::value;
    const int p = tid + sl * NTHREADS;
    const int r = p / TT, t = p - r * TT;
    const int v = (p < M::PAIRS) ? (3 * r * TT + t) * 4 : 0;
#pragma unroll
    for (int c = 0; c < 3; ++c)
      ck[sl][c] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rck, v, c * TT * 4, 0));
  });
}

// Flux backward for one RK stage (reference RHS, lib/models.py:130-150):
//   dS = -beta S I, dI = beta S I - gamma I, dR = gamma I  (+ fa_w * Fa for FaFp),
// masked where a state leaves (-1, 2); beta = |q0|, gamma = |q1|.  Writes the
// final-layer gradients (d q, d Fa incl. the |Fa| and posterior side-statistic
// terms) and applies the direct (d flux / d S, I) part of the RK adjoint.
template <class M, int SR>
__device__ __forceinline__ void flux_backward(float* lds, const KArgs& A, int n0, int jj, float dt,
                                              const float* ca, const float* cb, const float* mu, float cn) {
  constexpr int RG = (M::R + 3) / 4, ITEMS = TT * RG;
  constexpr int QO = M::HAS_P ? M::act_off(0, M::nl(0) - 1) : 0, QG = M::HAS_P ? M::gbuf(0, M::nl(0) - 1) : 0;
  constexpr int FO = M::HAS_A ? M::act_off(1, M::nl(1) - 1) : 0, FG = M::HAS_A ? M::gbuf(1, M::nl(1) - 1) : 0;
  constexpr bool VEC_Q = !M::HAS_P || M::QW <= M::kout(0, M::nl(0) - 1);
  constexpr bool VEC_F = !M::HAS_A || M::F4 <= M::kout(1, M::nl(1) - 1);
  // G regions per item: 4 (12 features, 8 rates: 16-B LDS ops), or all of them when R < 4 (one
  // item per trajectory with only its live features: at R = 1 a quarter of the VALU and LDS
  // work of a 4-region group, on the single wave that runs the pass)
  constexpr int G = M::R < 4 ? M::R : 4;
  constexpr int NQF = (3 * G + 3) / 4, NQR = (2 * G + 3) / 4;   // feature / rate quads per item
  constexpr int NF = 4 * NQF, NR = 4 * NQR;
  #pragma unroll 1
  for (int it = threadIdx.x; it < ITEMS; it += NTHREADS) {
    const int t = it & (TT - 1), rg = it >> 4;
    const bool valid = n0 + t < A.n_traj;
    float* rec = lds + t * SR;
    float Y[NF], dk[NF], dres[NF];
    const int f0 = 12 * rg;
    const int dko = jj == 3 ? M::RK_A : jj == 2 ? M::RK_DK3 : jj == 1 ? M::RK_DK2 : M::RK_DK1;
#pragma unroll
    for (int v = 0; v < NQF; ++v) {
      const f4 y = *reinterpret_cast<const f4*>(rec + M::Y_OFF + f0 + 4 * v);
      const f4 k = *reinterpret_cast<const f4*>(rec + dko + f0 + 4 * v);
#pragma unroll
      for (int e = 0; e < 4; ++e) { Y[4 * v + e] = y[e]; dk[4 * v + e] = k[e]; }
    }
    // the RK adjoint accumulators this stage updates, read with the other operands (every LDS
    // read of the item before its first write: one round trip)
    f4 ra[NQF], r1[NQF], r2[NQF], r3[NQF];
    if constexpr (M::HAS_P && !M::DYF) {
#pragma unroll
      for (int v = 0; v < NQF; ++v) {
        ra[v] = *reinterpret_cast<const f4*>(rec + M::RK_ACCY + f0 + 4 * v);
        r1[v] = *reinterpret_cast<const f4*>(rec + M::RK_DK1 + f0 + 4 * v);
        r2[v] = *reinterpret_cast<const f4*>(rec + M::RK_DK2 + f0 + 4 * v);
        r3[v] = *reinterpret_cast<const f4*>(rec + M::RK_DK3 + f0 + 4 * v);
      }
    }
    float qv[NR], fav[NF];
    if constexpr (M::HAS_P) {
#pragma unroll
      for (int v = 0; v < NQR; ++v) {
        const f4 x = *reinterpret_cast<const f4*>(rec + QO + 8 * rg + 4 * v);
#pragma unroll
        for (int e = 0; e < 4; ++e) qv[4 * v + e] = x[e];
      }
    }
    if constexpr (M::HAS_A) {
#pragma unroll
      for (int v = 0; v < NQF; ++v) {
        const f4 fa = *reinterpret_cast<const f4*>(rec + FO + f0 + 4 * v);
#pragma unroll
        for (int e = 0; e < 4; ++e) fav[4 * v + e] = fa[e];
      }
    }
    if (jj == 3) {
#pragma unroll
      for (int i = 0; i < NF; ++i) dk[i] = (dk[i] * 0.125f) * dt;
    }
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      const bool live = valid && i < 3 * G && (4 * rg + i / 3) < M::R;
      dres[i] = (!live || Y[i] > 2.f || Y[i] < -1.f) ? 0.f : dk[i];
    }
    if constexpr (M::HAS_A) {
      float dfa[NF];
#pragma unroll
      for (int i = 0; i < NF; ++i) {
        const bool live = valid && i < 3 * G && (4 * rg + i / 3) < M::R;
        const float d = M::HAS_P ? A.fa_w * dres[i] : dres[i];
        dfa[i] = live ? d + cn * fav[i] : 0.f;
      }
      if constexpr (VEC_F) {
#pragma unroll
        for (int v = 0; v < NQF; ++v) {
          f4 o = {dfa[4 * v], dfa[4 * v + 1], dfa[4 * v + 2], dfa[4 * v + 3]};
          *reinterpret_cast<f4*>(rec + FG + f0 + 4 * v) = o;
        }
      } else {
#pragma unroll
        for (int i = 0; i < NF; ++i)
          if (f0 + i < M::kout(1, M::nl(1) - 1)) rec[FG + f0 + i] = dfa[i];
      }
    }
    float dyf[NF];
#pragma unroll
    for (int i = 0; i < NF; ++i) dyf[i] = 0.f;
    if constexpr (M::HAS_P) {
      const float* q = qv;
      float dq[NR];
#pragma unroll
      for (int i = 0; i < NR; ++i) dq[i] = 0.f;
#pragma unroll
      for (int j = 0; j < G; ++j) {
        const bool live = valid && (4 * rg + j) < M::R;
        const float* y = Y + 3 * j;
        const float* dr = dres + 3 * j;
        const float q0 = q[2 * j], q1 = q[2 * j + 1];
        const float b = fabsf(q0), gm = fabsf(q1);
        const float dplus = dr[1] - dr[0];
        const float dminus = dr[2] - dr[1];
        const float dpi = dplus * y[1];                 // d(beta*S)
        float dbeta = dpi * y[0];
        dyf[3 * j] = dpi * b;
        dyf[3 * j + 1] = dplus * (b * y[0]) + dminus * gm;
        float dgam = dminus * y[1];
        if (live) {
          dbeta += ca[0] + cb[0] * (b - mu[0]);
          dgam += ca[1] + cb[1] * (gm - mu[1]);
        } else {
          dbeta = 0.f; dgam = 0.f;
        }
        dq[2 * j] = q0 > 0.f ? dbeta : (q0 < 0.f ? -dbeta : 0.f);
        dq[2 * j + 1] = q1 > 0.f ? dgam : (q1 < 0.f ? -dgam : 0.f);
      }
      if constexpr (VEC_Q) {
#pragma unroll
        for (int v = 0; v < NQR; ++v) {
          f4 o = {dq[4 * v], dq[4 * v + 1], dq[4 * v + 2], dq[4 * v + 3]};
          *reinterpret_cast<f4*>(rec + QG + 8 * rg + 4 * v) = o;
        }
      } else {
#pragma unroll
        for (int i = 0; i < NR; ++i)
          if (8 * rg + i < M::kout(0, M::nl(0) - 1)) rec[QG + 8 * rg + i] = dq[i];
      }
      // RK4 (3/8 rule) adjoint of the stage input, direct (flux) part; the MLP part
      // is added by mlp_backward's layer-0 epilogue (RkAdjointEp)
      //   Y2 = y + (dt k1)/3, Y3 = y + dt (k2 - k1/3), Y4 = y + dt (k1 - k2 + k3)
#pragma unroll
      for (int v = 0; v < NQF; ++v) {
        const f4 dY = {dyf[4 * v], dyf[4 * v + 1], dyf[4 * v + 2], dyf[4 * v + 3]};
        const int f = f0 + 4 * v;
        if constexpr (M::DYF) {
          // parked for the stage's one adjoint update (RkAdjointEp, with the MLP part)
          *reinterpret_cast<f4*>(rec + M::DYF_OFF + f) = dY;
          continue;
        }
        RkAdjointEp<M, SR>::rk_adjoint_update(dY, dt, jj, ra[v], r1[v], r2[v], r3[v],
                                              reinterpret_cast<f4*>(rec + M::RK_ACCY + f),
                                              reinterpret_cast<f4*>(rec + M::RK_DK1 + f),
                                              reinterpret_cast<f4*>(rec + M::RK_DK2 + f),
                                              reinterpret_cast<f4*>(rec + M::RK_DK3 + f));
      }
    }
    // the padded rows of the final-layer gradient slots (the slots alias wider layers'
    // gradients, so they are re-zeroed every stage), by the item of the last region group
    if (rg == RG - 1) {
      if constexpr (M::HAS_P) {
        constexpr int lo = cmin(8 * (RG - 1) + 4 * NQR, M::kout(0, M::nl(0) - 1)), hi = M::kout(0, M::nl(0) - 1);
#pragma unroll
        for (int o = lo; o < hi; o += 4) *reinterpret_cast<f4*>(rec + QG + o) = f4zero();
      }
      if constexpr (M::HAS_A) {
        constexpr int lo = cmin(12 * (RG - 1) + 4 * NQF, M::kout(1, M::nl(1) - 1)), hi = M::kout(1, M::nl(1) - 1);
#pragma unroll
        for (int o = lo; o < hi; o += 4) *reinterpret_cast<f4*>(rec + FG + o) = f4zero();
      }
    }
  }
}

// Tile end (deterministic RHS): per-trajectory layer-0 gradient sums -> global (the
// static-feature gradients are computed from them by ude_static_*_kernel); their trajectory
// sums -> the workgroup's bias row sums in LDS.
template <class M, int W, class AT>
__device__ __forceinline__ void g0_tile_end(const AT& A, float* lds, const f4* g0t, int tile, int lane) {
  const int t16 = lane & 15, g = lane >> 4;
  sfor<M::FT(0)>([&](auto kk) {
    constexpr int k = decltype(kk)::value;
    if constexpr (M::fowner(0, k) == W) {
      const f4 gv = g0t[M::nz_before(W, k)];
      if constexpr (M::HOIST) {
        float* dst = A.g0buf + ((size_t)tile * M::K0 + k * 16 + g * 4) * TT + t16;
        dst[0] = gv[0]; dst[TT] = gv[1]; dst[2 * TT] = gv[2]; dst[3 * TT] = gv[3];
      }
      f4 r = gv;
#pragma unroll
      for (int e = 0; e < 4; ++e) r[e] = row16_sum(r[e]);
      if (t16 == 0) {
        float* db = lds + M::DB_LDS + k * 16 + g * 4;
        db[0] += r[0]; db[1] += r[1]; db[2] += r[2]; db[3] += r[3];
      }
    }
  });
}

// Kernel end: wave W's dW register tiles (and BAYES eps-weighted ones) -> the workgroup slab.
template <class M, int W, class DW, class DS>
__device__ __forceinline__ void dw_to_slab(const DW& dw, const DS& dws, float* myslab, int lane) {
  sfor<M::D>([&](auto dd) {
    constexpr int d = decltype(dd)::value;
    sfor<M::FT(d)>([&](auto kk) {
      constexpr int k = decltype(kk)::value;
      if constexpr (M::fowner(d, k) == W) {
        constexpr int net = M::fnet(d, k);
        sfor<M::rti(net, d)>([&](auto cc) {
          constexpr int ct = decltype(cc)::value;
          reinterpret_cast<f4*>(myslab + (M::dyn_tiles_before(d, k) + ct) * 256)[lane] = dw[M::ndw_before(W, d, k) + ct];
          if constexpr (M::BAYES)
            reinterpret_cast<f4*>(myslab + M::SLAB_TOTAL + (M::dyn_tiles_before(d, k) + ct) * 256)[lane] =
                dws[M::ndw_before(W, d, k) + ct];
        });
      }
    });
  });
}

template <class M, int W>
__device__ void bwd_body(const KArgs& A, float* lds) {
  constexpr int SR = M::SR_B;
  constexpr int SL = M::SLOTS;
  constexpr int NDWn = M::NDW(W) > 0 ? M::NDW(W) : 1;
  constexpr int NZn = M::NZ(W) > 0 ? M::NZ(W) : 1;
  const int tid = threadIdx.x, lane = tid & 63;
  const int t16 = lane & 15, g = lane >> 4;
  const Sched sc(A.sched, A.n_steps, A.n_out);
  const size_t NRL = (size_t)A.n_traj * M::R * M::L;
  float* myslab = A.slab + (size_t)blockIdx.x * M::SLAB_STRIDE;
  const Rsrc rs = make_rsrc(A.pack, M::PACK_TOTAL * 4);

  // side-statistic cotangents -> per-eval gradient coefficients
  //   d mean_c / d p = 1/n ;  d std_c / d p = (p - mean_c) / ((n - 1) std_c)   (torch std backward)
  //   d |Fa| / d Fa = Fa / |Fa|  (0 when |Fa| == 0, torch norm backward)
  const double nev = 4.0 * (double)A.n_steps * (double)A.n_traj * (double)M::R;
  float ca[2] = {0.f, 0.f}, cb[2] = {0.f, 0.f}, mu[2] = {0.f, 0.f}, cn = 0.f;
  if constexpr (M::HAS_P) {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      mu[c] = A.st_mean[c];
      ca[c] = A.d_mean ? (float)((double)A.d_mean[c] / nev) : 0.f;
      const double sd = (double)A.st_std[c];
      cb[c] = A.d_std ? (float)((double)A.d_std[c] / ((nev - 1.0) * sd)) : 0.f;
    }
  }
  if constexpr (M::HAS_A) {
    const float nrm = A.st_norm[0];
    cn = (nrm > 0.f && A.d_norm) ? A.d_norm[0] / nrm : 0.f;
  }

  // SPLITB: the weight-gradient accumulators live on the partner waves (bwd_wbody / bwd_wbody_l)
  // GST: no weight-gradient accumulators (ude_gst_dw_kernel forms them from the stored rows)
  constexpr bool NO_DW = M::SPLITB || M::GST;
  f4 dw[NO_DW ? 1 : NDWn], dws[(M::BAYES && !M::GST) ? NDWn : 1], g0t[NZn], c1[NZn];
#pragma unroll
  for (int i = 0; i < (NO_DW ? 1 : NDWn); ++i) dw[i] = f4zero();
  if constexpr (M::BAYES && !M::GST) {
#pragma unroll
    for (int i = 0; i < NDWn; ++i) dws[i] = f4zero();
  }
  Prof prof_, *pf = nullptr;
#ifdef UDE_PROFILE
  if (A.prof && tid == 0) {
    pf = &prof_;
    for (int i = 0; i < NPROF; ++i) prof_.acc[i] = 0;
    prof_.last = __builtin_amdgcn_s_memtime();
  }
#endif

  WRegs<M, W, true> wr;
  wr.load(rs, lane);

  #pragma unroll 1
  for (int i = tid; i < M::LDS_B / 4; i += NTHREADS) lds[i] = 0.f;
  lds_sync();

  for (int tile = blockIdx.x; tile < A.n_tiles; tile += gridDim.x) {
    const int n0 = tile * TT;
    // the record's static features feed only the static hoist of a recomputed forward (and FULL0's
    // layer 0); with stored activations their alias of the activation region must stay untouched
    // (the SPLIT_BWD_L partner waves fill it by LDS-DMA meanwhile)
    if constexpr (!M::ACT_STORED || (M::FULL0 && !M::GST)) load_static<M, SR, M::XSB_OFF>(A.y0, lds, n0, A.n_traj);
    if constexpr (M::FULL0) {
      #pragma unroll 1
      for (int i = tid; i < TT * M::S16; i += NTHREADS) {
        const int t = i / M::S16, s = i - t * M::S16;
        lds[t * SR + M::DYS_OFF + s] = 0.f;
      }
    }
    // output cotangents of the last step: y_{n+1} share -> RK_A, y_n share staged in
    // DK3 (picked up by the step start).  Later steps get theirs under the flux pass
    // of the previous step's last stage.  (These pair-mapped stores are the only
    // writes of RK_A here: every (t, f < F) is covered, zeros without a step.)
    {
      float gv[SL][3], sg[SL][3], pg[SL][3];
      if (A.n_steps > 0) {
        out_issue<M>(A, sc, A.n_steps - 1, n0, gv);
        out_finish<M>(A, sc, A.n_steps - 1, n0, gv, sg, pg);
      } else {
#pragma unroll
        for (int sl = 0; sl < SL; ++sl)
#pragma unroll
          for (int c = 0; c < 3; ++c) { sg[sl][c] = 0.f; pg[sl][c] = 0.f; }
      }
      sfor<SL>([&](auto ss) {
        constexpr int sl = decltype(ss)::value;
        const int p = tid + sl * NTHREADS;
        if (p < M::PAIRS) {
          const int r = p / TT, t = p - r * TT;
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            lds[t * SR + M::RK_A + 3 * r + c] = sg[sl][c];
            lds[t * SR + M::RK_DK3 + 3 * r + c] = pg[sl][c];
          }
        }
      });
    }
    lds_sync();
    if constexpr (!M::ACT_STORED) static_hoist<M, W, SR, M::XSB_OFF>(rs, lds, c1, lane);
#pragma unroll
    for (int i = 0; i < NZn; ++i) g0t[i] = f4zero();
    lds_sync();
    UDE_STAMP(pf, 15);

    bool have_next = false;
    // small records with stored activations (CARRY): the next stage's activation rows and
    // checkpointed input are loaded into registers one whole stage ahead and written
    // straight into the record at that stage's start (no LDS staging slot, and the HBM
    // latency is covered by a full stage of work instead of one flux pass)
    constexpr bool CARRY = M::STORE_ACT && SL == 1;
    f4 actr[CARRY ? act_q_per_thread<M>() : 1];
    float ckr[SL][3];
    // CARRY: the next step's output cotangents are loaded at stage 1 of the step (a whole stage
    // ahead of the flux pass of stage 0 that consumes them)
    float gvc[SL][3];
    // GST: the next stage's checkpointed input and activation rows are carried in registers (no LDS
    // staging slot; the rows' HBM latency runs under the stage's four layer phases), and every phase's
    // input-gradient fragments are prefetched one phase ahead (mlp_backward PF)
    float ckg[M::GST ? SL : 1][3];
    constexpr bool GST_A = M::GST && M::STORE_ACT_D;
    f4 actg[GST_A ? act_q_per_thread<M>() : 1];
    float gvg[GST_A ? SL : 1][3];          // GST: the next step's output cotangents, loaded a stage ahead
    f4 fxp[(M::PF_X && M::WX_Q(W) > 0) ? M::WX_Q(W) : 1];
    for (int step = A.n_steps - 1; step >= 0; --step) {
      const float dt = sc.dt[step];
      // step start: RK_A already holds the adjoint of y_{n+1} including this step's
      // output cotangents (y_n-side share staged in DK3); set up the accumulators and
      // the stage cotangents of the 3/8 combination dy = (k1 + 3 (k2 + k3) + k4) dt / 8.
      {
        constexpr int NV = M::NVL;
        #pragma unroll 1
        for (int i = tid; i < TT * NV; i += NTHREADS) {
          const int t = i / NV, v = i - t * NV;
          float* rec = lds + t * SR + 4 * v;
          const f4 a = *reinterpret_cast<const f4*>(rec + M::RK_A);
          const f4 pend = *reinterpret_cast<const f4*>(rec + M::RK_DK3);
          const f4 sdk = (a * 0.125f) * dt;
          *reinterpret_cast<f4*>(rec + M::RK_PEND) = pend;
          *reinterpret_cast<f4*>(rec + M::RK_ACCY) = a;
          *reinterpret_cast<f4*>(rec + M::RK_DK1) = sdk;
          *reinterpret_cast<f4*>(rec + M::RK_DK2) = 3.0f * sdk;
          *reinterpret_cast<f4*>(rec + M::RK_DK3) = 3.0f * sdk;
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      UDE_STAMP(pf, 14);

      for (int jj = 3; jj >= 0; --jj) {
        // stage input: from the staging slot the previous stage's flux pass filled,
        // or (first stage of the tile) straight from the forward's checkpoint
        // large records: the step's output cotangents are loaded at its last stage's start, with
        // the activation rows (their latency is paid there anyway), not right before the flux pass
        float gvs[M::STORE_ACT_D ? SL : 1][3];
        if constexpr (M::STORE_ACT_D && !GST_A) {
          if (jj == 0 && step > 0) out_issue<M>(A, sc, step - 1, n0, gvs);
        }
        if (GST_A && have_next) {
          constexpr int QR = M::ACT_A4 / 4;
#pragma unroll
          for (int u = 0; u < act_q_per_thread<M>(); ++u) {
            const int i = tid + u * NTHREADS;
            if (i < TT * QR) {
              const int t = i / QR, q = i - t * QR;
              *reinterpret_cast<f4*>(lds + t * SR + M::ACT0 + 4 * q) = actg[GST_A ? u : 0];
            }
          }
        } else if constexpr (M::STORE_ACT_D && !M::SPLIT_BWD_L && UDE_ABL != 8) {
          // this stage's activation rows straight from the forward's store (issued first: the
          // stage-input copy below runs under their latency)
          constexpr int QR = M::ACT_A4 / 4;
          const f4* src = reinterpret_cast<const f4*>(act_block<M>(A.ckpt, A.n_tiles, A.n_steps, tile, step, jj));
          f4 av[act_q_per_thread<M>()];
#pragma unroll
          for (int u = 0; u < act_q_per_thread<M>(); ++u) {
            const int i = tid + u * NTHREADS;
            if (i < TT * QR) av[u] = src[act_src_q<M>(i)];
          }
#pragma unroll
          for (int u = 0; u < act_q_per_thread<M>(); ++u) {
            const int i = tid + u * NTHREADS;
            if (i < TT * QR) {
              const int t = i / QR, q = i - t * QR;
              *reinterpret_cast<f4*>(lds + t * SR + M::ACT0 + 4 * q) = av[u];
            }
          }
        }
        if constexpr (M::SPLIT_BWD) {
          // stage input, activation rows and output cotangents: the partner waves' (bwd_wbody)
        } else if constexpr (M::SPLIT_BWD_L) {
          // stage input and activation rows: the partner waves' (bwd_wbody_l)
        } else if (CARRY && have_next && UDE_ABL != 4) {
          constexpr int QR = M::ACT_A4 / 4;
#pragma unroll
          for (int u = 0; u < act_q_per_thread<M>(); ++u) {
            const int i = tid + u * NTHREADS;
            if (i < TT * QR) {
              const int t = i / QR, q = i - t * QR;
              *reinterpret_cast<f4*>(lds + t * SR + M::ACT0 + 4 * q) = actr[u];
            }
          }
          if (tid < M::PAIRS) {
            const int r = tid / TT, t = tid - r * TT;
#pragma unroll
            for (int c = 0; c < 3; ++c) lds[t * SR + M::Y_OFF + 3 * r + c] = ckr[0][c];
          }
        } else if (M::GST && have_next) {
          sfor<SL>([&](auto ss) {
            constexpr int sl = decltype(ss)::value;
            const int p = tid + sl * NTHREADS;
            if (p < M::PAIRS) {
              const int r = p / TT, t = p - r * TT;
#pragma unroll
              for (int c = 0; c < 3; ++c) lds[t * SR + M::Y_OFF + 3 * r + c] = ckg[M::GST ? sl : 0][c];
            }
          });
        } else if (have_next) {
          // the 3R stage-input features (quads of the F4-wide staging row, clipped to the
          // record's F16-wide Y slot: beyond it starts the activation region)
          constexpr int QY = cmin(M::F4, M::F16) / 4, NV = TT * QY;
          #pragma unroll 1
          for (int i = tid; i < NV; i += NTHREADS) {
            const int t = i / QY, v = i - t * QY;
            *reinterpret_cast<f4*>(lds + t * SR + M::Y_OFF + 4 * v) =
                *reinterpret_cast<const f4*>(lds + M::STG_LDS + t * M::F4 + 4 * v);
          }
          if constexpr (M::STORE_ACT) {
            constexpr int QR = M::ACT_A4 / 4;
            #pragma unroll
            for (int u = 0; u < act_q_per_thread<M>(); ++u) {
              const int i = tid + u * NTHREADS;
              if (i < TT * QR) {
                const int t = i / QR, q = i - t * QR;
                *reinterpret_cast<f4*>(lds + t * SR + M::ACT0 + 4 * q) =
                    *reinterpret_cast<const f4*>(lds + M::ACT_STG + 4 * i);
              }
            }
          }
        } else {
          if constexpr (M::STORE_ACT) {
            // first stage of the tile: its activations straight from the forward's store
            constexpr int QR = M::ACT_A4 / 4;
            const f4* src = reinterpret_cast<const f4*>(act_block<M>(A.ckpt, A.n_tiles, A.n_steps, tile, step, jj));
            #pragma unroll
            for (int u = 0; u < act_q_per_thread<M>(); ++u) {
              const int i = tid + u * NTHREADS;
              if (i < TT * QR) {
                const int t = i / QR, q = i - t * QR;
                *reinterpret_cast<f4*>(lds + t * SR + M::ACT0 + 4 * q) = src[act_src_q<M>(i)];
              }
            }
          }
          float ck[SL][3];
          ckpt_issue<M>(A, tile, step, jj, ck);
          sfor<SL>([&](auto ss) {
            constexpr int sl = decltype(ss)::value;
            const int p = tid + sl * NTHREADS;
            if (p < M::PAIRS) {
              const int r = p / TT, t = p - r * TT;
#pragma unroll
              for (int c = 0; c < 3; ++c) lds[t * SR + M::Y_OFF + 3 * r + c] = ck[sl][c];
            }
          });
        }
        UDE_STAMP(pf, 0);
        lds_sync();
        UDE_STAMP(pf, 1);
        // at the step's last stage the next step's output cotangents are loaded from
        // fwd phase 1 on (consumed after the flux pass)
        const int nstep = jj > 0 ? step : step - 1, njj = jj > 0 ? jj - 1 : 3;
        have_next = nstep >= 0;
        const bool next_out = jj == 0 && have_next;
        float gvn[SL][3];
        // BAYES: evaluation 4 step + jj's weight sample and eps
        Rsrc rse = rs, es = rs;
        if constexpr (M::BAYES) {
          const size_t ev = (size_t)(4 * step + jj);
          rse = make_rsrc(A.pack + ev * M::PACK_TOTAL, M::PACK_TOTAL * 4);
          es = make_rsrc(A.eslab + ev * M::SLAB_TOTAL, M::SLAB_TOTAL * 4);
        }
        if constexpr (M::PF_X) load_x_frags<M, W, M::D - 1>(rse, lane, fxp + M::xq_base(W, M::D - 1));
        // the next stage's checkpointed input: small records (one pair slot per thread)
        // fetch it before the recomputed forward, whose phases then hide the HBM latency;
        // wide ones under the flux pass (registers only live across that pass)
        float ckn[SL][3], sgn[SL][3], pgn[SL][3];
        constexpr bool EARLY_CK = SL == 1;
        if constexpr (M::SPLIT_BWD) {
          flux_backward<M, SR>(lds, A, n0, jj, dt, ca, cb, mu, cn);
        } else if constexpr (CARRY) {
          // the step's output cotangents (loaded a stage ago) are consumed before the next stage's
          // loads are issued: their wait sits in out_finish's runtime loop, where the compiler can
          // only emit vmcnt(0), which would also drain the fresh prefetch (HBM latency per step)
          if (next_out) out_finish<M>(A, sc, nstep, n0, gvc, sgn, pgn);
          if (jj == 1 && step > 0) out_issue<M>(A, sc, step - 1, n0, gvc);
          if (have_next) {
            ckpt_issue<M>(A, tile, nstep, njj, ckr);
            constexpr int QR = M::ACT_A4 / 4;
            const f4* src = reinterpret_cast<const f4*>(act_block<M>(A.ckpt, A.n_tiles, A.n_steps, tile, nstep, njj));
#pragma unroll
            for (int u = 0; u < act_q_per_thread<M>(); ++u) {
              const int i = tid + u * NTHREADS;
              if (i < TT * QR) actr[u] = src[act_src_q<M>(i)];
            }
          }
          if constexpr (UDE_ABL != 2) flux_backward<M, SR>(lds, A, n0, jj, dt, ca, cb, mu, cn);
        } else if (EARLY_CK && have_next) {
          ckpt_issue<M>(A, tile, nstep, njj, ckn);
        }
        if constexpr (CARRY) {
        } else if constexpr (M::STORE_ACT_D) {
          flux_backward<M, SR>(lds, A, n0, jj, dt, ca, cb, mu, cn);
        } else if constexpr (M::STORE_ACT) {
          // the stage's activations are the forward's (staged above); the next stage's are
          // fetched now and land in ACT_STG after the flux pass
          f4 actn[act_q_per_thread<M>()];
          if (have_next) {
            constexpr int QR = M::ACT_A4 / 4;
            const f4* src = reinterpret_cast<const f4*>(act_block<M>(A.ckpt, A.n_tiles, A.n_steps, tile, nstep, njj));
            #pragma unroll
            for (int u = 0; u < act_q_per_thread<M>(); ++u) {
              const int i = tid + u * NTHREADS;
              if (i < TT * QR) actn[u] = src[act_src_q<M>(i)];
            }
          }
          if (next_out) out_issue<M>(A, sc, nstep, n0, gvn);
          flux_backward<M, SR>(lds, A, n0, jj, dt, ca, cb, mu, cn);
          if (have_next) {
            constexpr int QR = M::ACT_A4 / 4;
            #pragma unroll
            for (int u = 0; u < act_q_per_thread<M>(); ++u) {
              const int i = tid + u * NTHREADS;
              if (i < TT * QR) *reinterpret_cast<f4*>(lds + M::ACT_STG + 4 * i) = actn[u];
            }
          }
        } else {
          mlp_forward<M, W, SR>(rse, lds, c1, lane, wr, pf, [&](auto dd) {
            if constexpr (decltype(dd)::value == (M::D > 2 ? 1 : 0))
              if (next_out) out_issue<M>(A, sc, nstep, n0, gvn);
          });
        }

        // flux backward: d k_j -> d q (pre-|.| rates), d Fa, and the direct d Y.
        // One item = one trajectory x a group of 4 regions (12 features, 8 rates):
        // every record access is a 16-B LDS op.
        if (!M::SPLIT_BWD_L && !GST_A && !EARLY_CK && have_next) ckpt_issue<M>(A, tile, nstep, njj, ckn);
        if constexpr (!M::ACT_STORED) flux_backward<M, SR>(lds, A, n0, jj, dt, ca, cb, mu, cn);
        UDE_STAMP(pf, 16);
        if (!M::SPLIT_BWD && next_out) {
          if constexpr (GST_A) out_finish<M>(A, sc, nstep, n0, gvg, sgn, pgn);
          else if constexpr (M::STORE_ACT_D) out_finish<M>(A, sc, nstep, n0, gvs, sgn, pgn);
          else if constexpr (!CARRY) out_finish<M>(A, sc, nstep, n0, gvn, sgn, pgn);
          // step nstep's output cotangents: the y_{n+1} share joins PEND (RK_A of the
          // next step = ACCY + PEND), the y_n share is staged in DK3 (dead at jj == 0)
          sfor<SL>([&](auto ss) {
            constexpr int sl = decltype(ss)::value;
            const int p = tid + sl * NTHREADS;
            if (p < M::PAIRS) {
              const int r = p / TT, t = p - r * TT;
#pragma unroll
              for (int c = 0; c < 3; ++c) {
                lds[t * SR + M::RK_PEND + 3 * r + c] += sgn[sl][c];
                lds[t * SR + M::RK_DK3 + 3 * r + c] = pgn[sl][c];
              }
            }
          });
        }
        UDE_STAMP(pf, 17);
        if constexpr (GST_A) {
          if (have_next) {
            // the next stage's input, activation rows and (a stage ahead of their consumer) output
            // cotangents, issued only after this stage's waits: no wait until the next stage start
            ckpt_issue<M>(A, tile, nstep, njj, ckg);
            const f4* src = reinterpret_cast<const f4*>(act_block<M>(A.ckpt, A.n_tiles, A.n_steps, tile, nstep, njj));
#pragma unroll
            for (int u = 0; u < act_q_per_thread<M>(); ++u) {
              const int i = tid + u * NTHREADS;
              if (i < TT * (M::ACT_A4 / 4)) actg[u] = src[act_src_q<M>(i)];
            }
            if (jj == 1 && step > 0) out_issue<M>(A, sc, step - 1, n0, gvg);
          }
        } else if (M::GST && !CARRY && have_next) {
#pragma unroll
          for (int sl = 0; sl < (M::GST ? SL : 1); ++sl)
#pragma unroll
            for (int c = 0; c < 3; ++c) ckg[sl][c] = ckn[sl][c];
        } else if (!CARRY && !M::SPLIT_BWD_L && have_next) {
          sfor<SL>([&](auto ss) {
            constexpr int sl = decltype(ss)::value;
            const int p = tid + sl * NTHREADS;
            if (p < M::PAIRS) {
              const int r = p / TT, t = p - r * TT;
#pragma unroll
              for (int c = 0; c < 3; ++c) lds[M::STG_LDS + t * M::F4 + 3 * r + c] = ckn[sl][c];
            }
          });
        }
        UDE_STAMP(pf, 18);
        UDE_STAMP(pf, 6);
        lds_sync();
        UDE_STAMP(pf, 11);
        if constexpr (UDE_ABL == 7) sfor<M::D>([&](auto) { lds_sync(); });
        else mlp_backward<M, W, SR, NO_DW, M::PF_X>(rse, es, lds, dw, dws, g0t, lane, pf,
                                           RkAdjointEp<M, SR>{lds + t16 * SR, dt, jj}, wr,
                                           M::GST ? A.gst + (((size_t)tile * A.n_steps + step) * 4 + jj) * TT * M::ACT_A4
                                                  : nullptr, fxp);
        if constexpr (M::SPLITX0) {
          // sum the waves' partial layer-0 input gradients -> RK adjoint (MLP part).  The RK rows
          // use the step-end thread <-> (t, quad) mapping, so the step end needs no barrier.
          auto x0sum = [&](int t, int f0) {
            const int m = f0 >> 4, li = ((f0 >> 2) & 3) * 16 + t;
            f4 v = f4zero();
#pragma unroll
            for (int w = 0; w < WAVES; ++w)
              v += *reinterpret_cast<const f4*>(lds + M::X0P_LDS + ((w * M::XT(0) + m) * 64 + li) * 4);
            return v;
          };
          constexpr int NV = M::NVL, NVX = cmin(M::F4, M::F16) / 4;
          #pragma unroll 1
          for (int i = tid; i < TT * NV; i += NTHREADS) {
            const int t = i / NV, v = i - t * NV;
            if (UDE_ABL != 5 && v < NVX) RkAdjointEp<M, SR>{lds + t * SR, dt, jj}(4 * v, x0sum(t, 4 * v));
          }
          if constexpr (M::FULL0) {
            constexpr int NS = M::S16 / 4;
            #pragma unroll 1
            for (int i = tid; i < TT * NS; i += NTHREADS) {
              const int t = i / NS, v = i - t * NS;
              RkAdjointEp<M, SR>{lds + t * SR, dt, jj}(M::F16 + 4 * v, x0sum(t, M::F16 + 4 * v));
            }
          }
        }

        UDE_STAMP(pf, 12);
      }
      // step end (same thread <-> element mapping as the step start: no barrier)
      {
        constexpr int NV = M::NVL;
        #pragma unroll 1
        for (int i = tid; i < TT * NV; i += NTHREADS) {
          const int t = i / NV, v = i - t * NV;
          float* rec = lds + t * SR + 4 * v;
          *reinterpret_cast<f4*>(rec + M::RK_A) =
              *reinterpret_cast<const f4*>(rec + M::RK_ACCY) + *reinterpret_cast<const f4*>(rec + M::RK_PEND);
        }
      }
      UDE_STAMP(pf, 13);
    }

    // ---- tile end: dy0 (dynamic), static-feature gradients, layer-0 bias sums ----
    lds_sync();
    #pragma unroll 1
    for (int p = tid; p < M::PAIRS; p += NTHREADS) {
      const int r = p / TT, t = p - r * TT;
      const int n = n0 + t;
      if (n < A.n_traj) {
        const size_t base = ((size_t)n * M::R + r) * M::L;
#pragma unroll
        for (int c = 0; c < 3; ++c)
          A.dy0[base + c] = lds[t * SR + M::RK_A + 3 * r + c] +
                            (A.dlatent ? A.dlatent[base + c] : A.dlat_sir[((size_t)n * M::R + r) * 3 + c]);
      }
    }
    if constexpr (M::FULL0) {
      // static latent dims: the summed input gradient of every evaluation (the direct cotangent of
      // every output time -- they are carried unchanged -- is added by ude_static_tsum_kernel, a
      // coalesced pass over d latent outside this latency-bound loop)
      #pragma unroll 1
      for (int i = tid; i < TT * M::S; i += NTHREADS) {
        const int t = i / M::S, s = i - t * M::S;
        const int n = n0 + t;
        if (n < A.n_traj) {
          const int r = s / (M::L - 3), c = 3 + s - r * (M::L - 3);
          A.dy0[((size_t)n * M::R + r) * M::L + c] = lds[t * SR + M::DYS_OFF + s];
        }
      }
    }
    lds_sync();
    // per-trajectory layer-0 gradient sums -> global (static-feature gradients are
    // computed from them by ude_static_*_kernel); their trajectory sums -> bias row sums
    // (BAYES: layer-0 bias and static columns were accumulated per evaluation instead)
    if constexpr (!M::BAYES && !M::SPLITB) g0_tile_end<M, W>(A, lds, g0t, tile, lane);
    lds_sync();
  }

  // ---- kernel end: register tiles + LDS row sums -> this workgroup's slab ----
  if constexpr (!NO_DW) dw_to_slab<M, W>(dw, dws, myslab, lane);
  // SPLITB: the partner waves' last bias row sums land before this barrier
  if constexpr (M::SPLITB) lds_sync();
  #pragma unroll 1
  for (int i = tid; i < (M::GST ? 0 : M::NDB); i += NTHREADS) {
    myslab[M::SLAB_DB + i] = lds[M::DB_LDS + i];
    if constexpr (M::BAYES) myslab[M::SLAB_TOTAL + M::SLAB_DB + i] = lds[M::DBS_LDS + i];
  }
#ifdef UDE_PROFILE
  if (pf) for (int i = 0; i < NPROF; ++i) A.prof[(size_t)blockIdx.x * NPROF + i] = prof_.acc[i];
#endif
}
// L = 8, 16-B aligned rows: one thread per (n, r) row, whole 32-B rows loaded (both 16-B halves of every
// output time in flight at once, coalesced), the same additions in the same order as the scalar kernel
// below (dy0 first, then output times ascending): bitwise the same dy0.
template <class M>
__global__ __launch_bounds__(256) void ude_static_tsum_rows_kernel(const float* __restrict__ dlatent, int n_traj,
                                                                   int n_times, float* __restrict__ dy0) {
  static_assert(M::L == 8, "row kernel: L = 8");
  const size_t NR = (size_t)n_traj * M::R, NRL = NR * M::L;
  for (size_t nr = (size_t)blockIdx.x * 256 + threadIdx.x; nr < NR; nr += (size_t)gridDim.x * 256) {
    f4* d = reinterpret_cast<f4*>(dy0 + nr * M::L);
    f4 lo = d[0], hi = d[1];
    float v3 = lo[3];
    #pragma unroll 3
    for (int jt = 0; jt < n_times; ++jt) {
      const f4* g = reinterpret_cast<const f4*>(dlatent + (size_t)jt * NRL + nr * M::L);
      v3 += g[0][3];
      hi += g[1];
    }
    lo[3] = v3;
    d[0] = lo;
    d[1] = hi;
  }
}

// FULL0 (Bayesian RHS, static dims in the solve's layer 0): dy0[n, r, c >= 3] += sum_j dlatent[j, n, r, c]
// in output order j (the same additions as one loop after the input-gradient sum).
template <class M>
__global__ __launch_bounds__(256) void ude_static_tsum_kernel(const float* __restrict__ dlatent, int n_traj,
                                                              int n_times, float* __restrict__ dy0) {
  constexpr int SPR = M::L - 3;
  const size_t NRL = (size_t)n_traj * M::R * M::L, total = (size_t)n_traj * M::R * SPR;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
    const size_t nr = i / SPR;
    const size_t base = nr * M::L + 3 + (i - nr * SPR);
    float v = dy0[base];
    #pragma unroll 4
    for (int jt = 0; jt < n_times; ++jt) v += dlatent[(size_t)jt * NRL + base];
    dy0[base] = v;
  }
}

// SPLIT_BWD partner wave W + 4: the weight gradients of every stage (mlp_backward_dw), on the
// exact barrier sequence of bwd_body's critical-path waves (every lds_sync there has its
// counterpart here, in the same order).
template <class M, int W>
__device__ void bwd_wbody(const KArgs& A, float* lds) {
  constexpr int SR = M::SR_B;
  constexpr int NDWn = M::NDW(W) > 0 ? M::NDW(W) : 1;
  constexpr int NZn = M::NZ(W) > 0 ? M::NZ(W) : 1;
  constexpr int NGn = M::NG(W) > 0 ? M::NG(W) : 1;
  const int lane = threadIdx.x & 63, t16 = lane & 15, g = lane >> 4;
  float* myslab = A.slab + (size_t)blockIdx.x * M::SLAB_STRIDE;
  f4 dw[NDWn], g0t[NZn], gacc[NGn];
#pragma unroll
  for (int i = 0; i < NDWn; ++i) dw[i] = f4zero();
#pragma unroll
  for (int i = 0; i < NGn; ++i) gacc[i] = f4zero();
  __builtin_amdgcn_s_setprio(1);         // as bwd_wbody_l (M1 bwd 4.44 -> 4.38 ms, profiles/r05/ab_partner_prio_m1.txt)
  lds_sync();                            // record zeroed
  // These waves also move the stage data (the critical-path waves issue no global load in the
  // stage loop): each stage's checkpointed input and activation rows, loaded one stage ahead into
  // registers and written into the record at the stage start, and the output cotangents of each
  // step, loaded a stage ahead and folded into the RK adjoint rows.  Their waits are this wave's
  // own, so no wait of the critical path can drain the prefetch.
  const Sched sc(A.sched, A.n_steps, A.n_out);
  const int wt = threadIdx.x - NTHREADS;                // 0..255: the pair / quad index
  constexpr int QR = M::ACT_A4 / 4, NQ = act_q_per_thread<M>();
  f4 actr[NQ];
  float ckr[1][3], gvc[1][3];
  auto put_stage = [&](int tile_) {                     // carried rows -> the record
#pragma unroll
    for (int u = 0; u < NQ; ++u) {
      const int i = wt + u * NTHREADS;
      if (i < TT * QR) {
        const int t = i / QR, q = i - t * QR;
        *reinterpret_cast<f4*>(lds + t * SR + M::ACT0 + 4 * q) = actr[u];
      }
    }
    if (wt < M::PAIRS) {
      const int r = wt / TT, t = wt - r * TT;
#pragma unroll
      for (int c = 0; c < 3; ++c) lds[t * SR + M::Y_OFF + 3 * r + c] = ckr[0][c];
    }
  };
  auto get_stage = [&](int tile_, int step_, int jj_) {  // issue one stage's loads
    ckpt_issue<M>(A, tile_, step_, jj_, ckr, wt);
    const f4* src = reinterpret_cast<const f4*>(act_block<M>(A.ckpt, A.n_tiles, A.n_steps, tile_, step_, jj_));
#pragma unroll
    for (int u = 0; u < NQ; ++u) {
      const int i = wt + u * NTHREADS;
      if (i < TT * QR) actr[u] = src[act_src_q<M>(i)];
    }
  };
  for (int tile = blockIdx.x; tile < A.n_tiles; tile += gridDim.x) {
    const int n0 = tile * TT;
    lds_sync();                          // last step's output cotangents staged
#pragma unroll
    for (int i = 0; i < NZn; ++i) g0t[i] = f4zero();
    lds_sync();
    bool have = false;
    for (int step = A.n_steps - 1; step >= 0; --step) {
      #pragma unroll 1
      for (int jj = 3; jj >= 0; --jj) {
        const int nstep = jj > 0 ? step : step - 1, njj = jj > 0 ? jj - 1 : 3;
        if (!have) get_stage(tile, step, jj);           // the tile's first stage
        put_stage(tile);
        lds_sync();                      // stage input + activation rows in the record
        // the rest runs in the flux interval (these waves' MFMA-free wait), not ahead of the
        // stage-input barrier, where its dependent scalar schedule loads delayed the critical path
        if (jj == 0 && nstep >= 0) {
          // step nstep's output cotangents: the y_{n+1} share joins PEND (RK_A of the next step
          // = ACCY + PEND), the y_n share is staged in DK3 (dead at jj == 0; read at the step start)
          float sg[1][3], pg[1][3];
          out_finish<M>(A, sc, nstep, n0, gvc, sg, pg, wt);
          if (wt < M::PAIRS) {
            const int r = wt / TT, t = wt - r * TT;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
              lds[t * SR + M::RK_PEND + 3 * r + c] += sg[0][c];
              lds[t * SR + M::RK_DK3 + 3 * r + c] = pg[0][c];
            }
          }
        }
        if (jj == 1 && step > 0) out_issue<M>(A, sc, step - 1, n0, gvc, wt);
        have = nstep >= 0;
        if (have) get_stage(tile, nstep, njj);
        lds_sync();                      // flux pass: final-layer gradients written
        if constexpr (UDE_ABL == 1) { sfor<M::D>([&](auto) { lds_sync(); }); }
        else mlp_backward_dw<M, W, SR>(lds, dw, g0t, gacc, lane);
      }
    }
    lds_sync();                          // tile end: dy0
    lds_sync();
    g0_tile_end<M, W>(A, lds, g0t, tile, lane);
    lds_sync();
  }
  // kernel end: dW tiles -> slab; bias row sums of layers >= 1 from the per-trajectory sums
  f4 none[1];
  dw_to_slab<M, W>(dw, none, myslab, lane);
  sfor<M::D>([&](auto dd) {
    constexpr int d = decltype(dd)::value;
    if constexpr (d > 0) sfor<M::FT(d)>([&](auto kk) {
      constexpr int k = decltype(kk)::value;
      if constexpr (M::fowner(d, k) == W) {
        f4 r = gacc[M::ng_before(W, d, k)];
#pragma unroll
        for (int e = 0; e < 4; ++e) r[e] = row16_sum(r[e]);
        if (t16 == 0) {
          float* db = lds + M::DB_LDS + (M::FTbase(d) + k) * 16 + g * 4;
          db[0] += r[0]; db[1] += r[1]; db[2] += r[2]; db[3] += r[3];
        }
      }
    });
  });
  lds_sync();                            // bias row sums complete -> bwd_body copies them
}


// ---- SPLIT_BWD_L: the partner waves of large records ------------------------------------
// Barrier for waves with LDS-DMA loads in flight: their LDS writes are retired by lgkmcnt, the
// DMA (which counts on vmcnt) stays in flight across it (lds_sync's release fence would drain it,
// holding the critical-path waves at this barrier for the HBM latency).
__device__ __forceinline__ void lds_sync_dma() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_waitcnt(0xC07F);          // lgkmcnt(0) only
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ void wait_dma() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_waitcnt(0x0F70);          // vmcnt(0)
  __builtin_amdgcn_sched_barrier(0);
}
typedef __attribute__((address_space(3))) void* LdsPtr;

// LDS-DMA of one layer's activation rows (net, i) of tile-stage (step, jj) into the record:
// partner wave W moves trajectories 4W .. 4W+3, one 16-B-per-lane instruction each (kout / 4
// lanes; the record row's layer slice is contiguous, so the lane-linear destination fits).  The
// source goes through a buffer resource: SGPR base of the tile-stage block, one shared per-lane
// offset (16 lane) and the slice's constant offset in the scalar soffset.  Per-instruction
// per-lane addresses held in VGPRs spilled, and every spill reload (a vmcnt wait) drained all
// DMAs in flight.
template <class M, int W, int net, int i>
__device__ __forceinline__ void dma_layer(Rsrc src, float* lds, int lane) {
  if constexpr (UDE_ABL == 22) return;
  constexpr int SR = M::SR_B, KO = M::kout(net, i), OFF = M::act_off(net, i);
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int t = 4 * W + u;
#if defined(__HIP_DEVICE_COMPILE__)
    if (lane < KO / 4)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(src, (LdsPtr)(lds + t * SR + OFF), 16, 16 * lane,
                                               (t * M::XST_W + M::ACT_IN + (OFF - M::ACT0)) * 4, 0, 0);
#endif
  }
}
template <class M>
__device__ __forceinline__ Rsrc act_rsrc(const KArgs& A, int tile, int step, int jj) {
  return make_rsrc(act_block<M>(A.ckpt, A.n_tiles, A.n_steps, tile, step, jj), TT * M::XST_W * 4);
}
// the layers whose last reader of the current stage is phase d (d = D: the flux pass)
template <class M, int W, int d>
__device__ __forceinline__ void dma_freed(Rsrc src, float* lds, int lane) {
  sfor<2>([&](auto nn) {
    constexpr int net = decltype(nn)::value;
    if constexpr (d == M::D) {
      if constexpr (M::has(net, 0)) dma_layer<M, W, net, M::nl(net) - 1>(src, lds, lane);
    } else if constexpr (d >= 1 && M::has(net, d) && d - 1 < M::nl(net) - 1) {
      dma_layer<M, W, net, d - 1>(src, lds, lane);
    }
  });
}
// LDS-DMA of the checkpointed stage input ([F][16], contiguous) into the staging slot
template <class M, int W>
__device__ __forceinline__ void dma_ckpt(const KArgs& A, float* lds, int tile, int step, int jj, int lane) {
  constexpr int NF = M::F * TT, NC = (NF + 255) / 256;
  const Rsrc src = make_rsrc(A.ckpt + ckpt_index(tile, A.n_steps, step, jj, M::F, 0, 0), NF * 4);
#pragma unroll
  for (int c = W; c < NC; c += WAVES) {
#if defined(__HIP_DEVICE_COMPILE__)
    if (c * 256 + 4 * lane < NF)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(src, (LdsPtr)(lds + M::STG_LDS + c * 256), 16, 16 * lane, c * 1024,
                                               0, 0);
#endif
  }
}

// Weight gradients of one stage (large records): as mlp_backward_dw, with each owned tile's input
// operands read in chunks of XC column tiles (registers: the dW accumulators fill this wave) and the
// bias sums reduced across the tile's trajectories into the LDS row sums every phase.
template <class M, int W, int SR, class After>
__device__ __forceinline__ void mlp_backward_dw_l(float* lds, f4* dw, f4* g0t, int lane, const After& after,
                                                  Prof* pf = nullptr) {
  const int t = lane & 15, g = lane >> 4;
  const float* rec = lds + t * SR;
  constexpr int XC = 4;
  sfor<M::D>([&](auto ee) {
    constexpr int d = M::D - 1 - decltype(ee)::value;
    sfor<M::FT(d)>([&](auto kk) {
      constexpr int k = decltype(kk)::value;
      if constexpr (M::fowner(d, k) == W) {
        constexpr int net = M::fnet(d, k), rt = M::frt(d, k), goff = M::gbuf(net, d);
        constexpr int inoff = d == 0 ? M::Y_OFF : M::act_off(net, d - 1);
        constexpr int NC = M::rti(net, d);
        const f4 gv = *reinterpret_cast<const f4*>(rec + goff + rt * 16 + g * 4);
        float ga[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) ga[s] = lds[(4 * g + s) * SR + goff + rt * 16 + t];
        if constexpr (UDE_ABL != 21) sfor<(NC + XC - 1) / XC>([&](auto cc0) {
          constexpr int c0 = decltype(cc0)::value * XC;
          constexpr int NCC = cmin(XC, NC - c0);
          float bv[4][NCC];
#pragma unroll
          for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int ct = 0; ct < NCC; ++ct) bv[s][ct] = lds[(4 * g + s) * SR + inoff + (c0 + ct) * 16 + t];
#pragma unroll
          for (int s = 0; s < 4; ++s)
            sfor<NCC>([&](auto cc) {
              constexpr int ct = decltype(cc)::value;
              constexpr int idx = M::ndw_before(W, d, k) + c0 + ct;
              dw[idx] = mfma4(ga[s], bv[s][ct], dw[idx]);
            });
        });
        if constexpr (d == 0) {
          g0t[M::nz_before(W, k)] += gv;
        } else {
          f4 r = gv;
#pragma unroll
          for (int e = 0; e < 4; ++e) r[e] = row16_sum(r[e]);
          if (t == 0) {
            float* db = lds + M::DB_LDS + (M::FTbase(d) + k) * 16 + g * 4;
            db[0] += r[0]; db[1] += r[1]; db[2] += r[2]; db[3] += r[3];
          }
        }
      }
    });
    // the next stage's rows freed by phase d + 1 (D: the flux pass) are fetched behind this phase's
    // MFMAs instead of ahead of them, except layer 0's (needed soonest: issued as phase 0 starts)
    if constexpr (d + 1 >= 2) after(std::integral_constant<int, d + 1>{});
    UDE_STAMP(pf, 20 + d);
    lds_sync_dma();
    UDE_STAMP(pf, 7 + d);
    if constexpr (d == 1) after(std::integral_constant<int, 1>{});
    UDE_STAMP(pf, 24 + d);
  });
}

// SPLIT_BWD_L partner wave W + 4: weight gradients of every stage and the next stage's data
// (LDS-DMA), on the exact barrier sequence of bwd_body's critical-path waves.
template <class M, int W>
__device__ void bwd_wbody_l(const KArgs& A, float* lds) {
  constexpr int SR = M::SR_B;
  constexpr int NDWn = M::NDW(W) > 0 ? M::NDW(W) : 1;
  constexpr int NZn = M::NZ(W) > 0 ? M::NZ(W) : 1;
  int lane = threadIdx.x & 63;
  float* myslab = A.slab + (size_t)blockIdx.x * M::SLAB_STRIDE;
  f4 dw[NDWn], g0t[NZn];
#pragma unroll
  for (int i = 0; i < NDWn; ++i) dw[i] = f4zero();
  // the second-dispatched half of the workgroup at static priority 1 for the whole launch (the
  // arbitration loser otherwise; MI355X_MICROARCH "Two waves per SIMD" item 4): state49 bwd
  // 1.744 -> 1.724 ms (profiles/r05/ab_partner_prio.txt)
  __builtin_amdgcn_s_setprio(1);
  Prof prof_, *pf = nullptr;
#if defined(UDE_PROFILE) && defined(UDE_PROFILE_PARTNER)
  // diagnostic (-DUDE_PROFILE_PARTNER on top of -DUDE_PROFILE): partner wave 4 (W = 0) stamps its own
  // segments into row 2 * PROF_FWD_SLOT + block.  Its stamps perturb the stage far more than the
  // critical path's (s_memtime waits on the partner's LDS traffic): a separate build, for its shares.
  if (W == 0 && A.prof && lane == 0) {
    pf = &prof_;
    for (int i = 0; i < NPROF; ++i) prof_.acc[i] = 0;
    prof_.last = __builtin_amdgcn_s_memtime();
  }
#endif
  lds_sync();                                           // record zeroed
  // staged stage input [f][t] -> Y slot [t][f]: each wave moves exactly the 256-float chunks its own
  // dma_ckpt wrote (its vmcnt wait covers only its own DMAs; the other waves' may still be landing)
  auto put_stage = [&]() {
    constexpr int NF = M::F * TT, NC = (NF + 255) / 256;
#pragma unroll
    for (int c = W; c < NC; c += WAVES)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int i = c * 256 + e * 64 + lane;
        if (i < NF) lds[(i & 15) * SR + M::Y_OFF + (i >> 4)] = lds[M::STG_LDS + i];
      }
  };
  auto dma_all = [&](int tile_, int step_, int jj_) {
    const Rsrc src = act_rsrc<M>(A, tile_, step_, jj_);
    sfor<2>([&](auto nn) {
      constexpr int net = decltype(nn)::value;
      sfor<M::nl(net)>([&](auto ii) { dma_layer<M, W, net, decltype(ii)::value>(src, lds, lane); });
    });
    dma_ckpt<M, W>(A, lds, tile_, step_, jj_, lane);
  };
  for (int tile = blockIdx.x; tile < A.n_tiles; tile += gridDim.x) {
    // the tile's first stage: everything at once (nothing of it is in the record yet)
    if (A.n_steps > 0) dma_all(tile, A.n_steps - 1, 3);
    lds_sync_dma();                                     // last step's output cotangents staged
#pragma unroll
    for (int i = 0; i < NZn; ++i) g0t[i] = f4zero();
    lds_sync_dma();
    for (int step = A.n_steps - 1; step >= 0; --step) {
      #pragma unroll 1
      for (int jj = 3; jj >= 0; --jj) {
        const int nstep = jj > 0 ? step : step - 1, njj = jj > 0 ? jj - 1 : 3;
        const bool have = nstep >= 0;
        // lane is opaque per stage: the ~40 lane-derived LDS addresses of the stage (staging copy,
        // operand reads) are recomputed here instead of hoisted out of the loop, where they spilled
        // next to the 176 dW VGPRs and every scratch reload (a vmcnt wait) drained the DMAs in flight
        asm volatile("" : "+v"(lane));
        UDE_STAMP(pf, 13);
        wait_dma();                                     // this stage's rows and input have landed
        UDE_STAMP(pf, 0);
        put_stage();
        UDE_STAMP(pf, 2);
        lds_sync_dma();                                 // stage input + activation rows in the record
        UDE_STAMP(pf, 1);
        if (have) dma_ckpt<M, W>(A, lds, tile, nstep, njj, lane);   // staging slot free again
        UDE_STAMP(pf, 3);
        lds_sync_dma();                                 // flux pass: final-layer gradients written
        UDE_STAMP(pf, 16);
        UDE_STAMP(pf, 17);
        mlp_backward_dw_l<M, W, SR>(lds, dw, g0t, lane, [&](auto dd) {
          constexpr int d = decltype(dd)::value;
          if constexpr (d >= 1)
            if (have) dma_freed<M, W, d>(act_rsrc<M>(A, tile, nstep, njj), lds, lane);
        }, pf);
      }
    }
    lds_sync_dma();                                     // tile end: dy0
    lds_sync_dma();
    g0_tile_end<M, W>(A, lds, g0t, tile, lane);
    lds_sync_dma();
    UDE_STAMP(pf, 15);
  }
  wait_dma();
  f4 none[1];
  dw_to_slab<M, W>(dw, none, myslab, lane);
  lds_sync();                                           // bias row sums complete -> bwd_body copies them
#ifdef UDE_PROFILE
  if (pf) for (int i = 0; i < NPROF; ++i) A.prof[(size_t)(2 * PROF_FWD_SLOT + blockIdx.x) * NPROF + i] = prof_.acc[i];
#endif
}

template <class M>
__global__ __launch_bounds__(M::BWD_THREADS) void ude_bwd_kernel(KArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if constexpr (M::SPLIT_BWD) {
    if (w >= WAVES) {
      if (w == 4) bwd_wbody<M, 0>(a, lds);
      else if (w == 5) bwd_wbody<M, 1>(a, lds);
      else if (w == 6) bwd_wbody<M, 2>(a, lds);
      else bwd_wbody<M, 3>(a, lds);
      return;
    }
  }
  if constexpr (M::SPLIT_BWD_L) {
    if (w >= WAVES) {
      if (w == 4) bwd_wbody_l<M, 0>(a, lds);
      else if (w == 5) bwd_wbody_l<M, 1>(a, lds);
      else if (w == 6) bwd_wbody_l<M, 2>(a, lds);
      else bwd_wbody_l<M, 3>(a, lds);
      return;
    }
  }
  if (w == 0) bwd_body<M, 0>(a, lds);
  else if (w == 1) bwd_body<M, 1>(a, lds);
  else if (w == 2) bwd_body<M, 2>(a, lds);
  else bwd_body<M, 3>(a, lds);
}

// ============================================================================
// Weight packing (one launch, blockIdx.y = segment)
// ============================================================================
struct PackPtrs {
  const float* W[2][5];
  const float* b[2][5];
  const float* Ws[2][5];   // BAYES: w_std / b_std (|.| is taken here, models_bayes.py:45-46)
  const float* bs[2][5];
  const float* eps;        // BAYES: [eval][N_PARAMS] in torch parameter order
};

template <class M>
__device__ __forceinline__ int static_col(int s) {
  const int r = s / (M::L - 3);
  return r * M::L + 3 + (s - r * (M::L - 3));
}

// One launch packs every segment (blockIdx.y) of one weight set; BAYES: blockIdx.z =
// evaluation, whose sample w = mu + eps * |std| (the reference's fp32 op order) is
// packed PACK_TOTAL floats after the previous one's.
template <class M>
__global__ __launch_bounds__(256) void ude_pack_kernel(PackPtrs P, float* __restrict__ pack) {
  const int seg = blockIdx.y;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  const size_t ev = M::BAYES ? blockIdx.z : 0;
  pack += ev * M::PACK_TOTAL;
  sfor<2>([&](auto nn) {
    constexpr int net = decltype(nn)::value;
    sfor<5>([&](auto ii) {
      constexpr int i = decltype(ii)::value;
      if constexpr (M::has(net, i)) {
        constexpr int base = (net * 5 + i) * 3;
        constexpr int in = M::in_dim(net, i), out = M::out_dim(net, i);
        constexpr int in_full = i == 0 ? M::R * M::L : in;
        const float* Wp = P.W[net][i];
        auto wval = [&](int o, int f) -> float {
          const int col = i == 0 ? M::col0(f) : (f < in ? f : -1);
          if (o >= out || col < 0) return 0.f;
          const size_t w = (size_t)o * in_full + col;
          float v = Wp[w];
          if constexpr (M::BAYES) v = v + P.eps[ev * M::N_PARAMS + M::param_w_off(net, i) + w] * fabsf(P.Ws[net][i][w]);
          return v;
        };
        if (seg == base + 0 && idx < M::wf_size(net, i)) {
          constexpr int KQ = M::kin(net, i) / 4, NQ = M::kin(net, i) / 16;
          const int e = idx & 3, ln = (idx >> 2) & 63, q = (idx >> 8) % NQ, rt = (idx >> 8) / NQ;
          pack[M::wf_off(net, i) + idx] = wval(rt * 16 + (ln & 15), (ln >> 4) * KQ + 4 * q + e);
        } else if (seg == base + 1 && idx < M::wt_size(net, i)) {
          constexpr int KQ = M::kout(net, i) / 4, NQ = M::kout(net, i) / 16;
          const int e = idx & 3, ln = (idx >> 2) & 63, q = (idx >> 8) % NQ, rt = (idx >> 8) / NQ;
          pack[M::wt_off(net, i) + idx] = wval((ln >> 4) * KQ + 4 * q + e, rt * 16 + (ln & 15));
        } else if (seg == base + 2 && idx < M::b_size(net, i)) {
          float v = 0.f;
          if (idx < out) {
            v = P.b[net][i][idx];
            if constexpr (M::BAYES)
              v = v + P.eps[ev * M::N_PARAMS + M::param_w_off(net, i) + out * in_full + idx] * fabsf(P.bs[net][i][idx]);
          }
          pack[M::b_off(net, i) + idx] = v;
        }
      }
    });
    if constexpr (M::HOIST && M::has(net, 0)) {
      if (seg == 30 + net && idx < M::wsf_size(net)) {
        constexpr int KQ = M::S16 / 4, NQ = M::S16 / 16;
        constexpr int out = M::out_dim(net, 0);
        const int e = idx & 3, ln = (idx >> 2) & 63, q = (idx >> 8) % NQ, rt = (idx >> 8) / NQ;
        const int o = rt * 16 + (ln & 15), s = (ln >> 4) * KQ + 4 * q + e;
        pack[M::wsf_off(net) + idx] =
            (o < out && s < M::S) ? P.W[net][0][(size_t)o * M::R * M::L + static_col<M>(s)] : 0.f;
      }
    }
  });
  if constexpr (M::HOIST) {
    if (seg == 32 && idx < M::W0SP_SIZE) {
      // plain [merged layer-0 row][static feature] copy (dy0 static kernel)
      int om = idx / M::S16;
      const int s = idx - om * M::S16;
      int net = 0;
      if (!M::HAS_P || om >= (M::HAS_P ? M::kout(0, 0) : 0)) {
        net = 1;
        om -= M::HAS_P ? M::kout(0, 0) : 0;
      }
      const int out = M::out_dim(net, 0);
      float v = 0.f;
      if (s < M::S && om < out && (net == 0 ? M::HAS_P : M::HAS_A))
        v = P.W[net][0][(size_t)om * M::R * M::L + static_col<M>(s)];
      pack[M::W0SP_OFF + idx] = v;
    }
  }
}

// Decoder Linear(3R -> R) (lib/models.py:39) -> the DEC epilogue's fragment layout (Model::DEC_PACK).
template <class M>
__global__ __launch_bounds__(256) void ude_dec_pack_kernel(const float* __restrict__ Wd, const float* __restrict__ bd,
                                                           float* __restrict__ out) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx < M::DEC_WF) {
    constexpr int KQ = M::F16 / 4, NQ = M::F16 / 16;
    const int e = idx & 3, ln = (idx >> 2) & 63, q = (idx >> 8) % NQ, rt = (idx >> 8) / NQ;
    const int o = rt * 16 + (ln & 15), f = (ln >> 4) * KQ + 4 * q + e;
    out[idx] = (o < M::R && f < M::F) ? Wd[(size_t)o * M::F + f] : 0.f;
  } else if (idx < M::DEC_PACK) {
    const int o = idx - M::DEC_WF;
    out[idx] = o < M::R ? bd[o] : 0.f;
  }
}

// ============================================================================
// Deterministic reductions over the per-workgroup partials
// ============================================================================
// Slab offset -> index into the torch-ordered parameter vector (-1: padding).
// Inverse of the dW tile layout: tile T = dyn_tiles_before(d, k) + ct holds rows
// frt(d, k) * 16 + [0, 16) of layer d of net fnet(d, k) and input columns ct * 16 +
// [0, 16) in MFMA C order (lane = (row >> 2) * 16 + col, reg = row & 3).
template <class M>
__device__ __forceinline__ int slab_to_param(int off) {
  int e = -1;
  if (off >= M::SLAB_DB) {
    const int idx = off - M::SLAB_DB, T = idx >> 4, row = idx & 15;
    sfor<M::D>([&](auto ii) {
      constexpr int i = decltype(ii)::value;
      if (T >= M::FTbase(i) && T < M::FTbase(i) + M::FT(i)) {
        const int k = T - M::FTbase(i);
        sfor<2>([&](auto nn) {
          constexpr int net = decltype(nn)::value;
          if constexpr (M::has(net, i)) {
            constexpr int kb = net == 0 ? 0 : M::rto(0, i);
            constexpr int in_full = i == 0 ? M::R * M::L : M::in_dim(net, i);
            if (k >= kb && k < kb + M::rto(net, i)) {
              const int o = (k - kb) * 16 + row;
              if (o < M::out_dim(net, i)) e = M::param_w_off(net, i) + M::out_dim(net, i) * in_full + o;
            }
          }
        });
      }
    });
    return e;
  }
  const int T = off >> 8, wq = off & 255, ln = wq >> 2;
  const int row = (ln >> 4) * 4 + (wq & 3), fc = ln & 15;
  sfor<M::D>([&](auto ii) {
    constexpr int i = decltype(ii)::value;
    sfor<M::FT(i)>([&](auto kk) {
      constexpr int k = decltype(kk)::value;
      constexpr int net = M::fnet(i, k);
      constexpr int t0 = M::dyn_tiles_before(i, k);
      if (T >= t0 && T < t0 + M::rti(net, i)) {
        const int f = (T - t0) * 16 + fc;
        const int o = M::frt(i, k) * 16 + row;
        constexpr int in_full = i == 0 ? M::R * M::L : M::in_dim(net, i);
        const int col = i == 0 ? M::col0(f) : (f < M::in_dim(net, i) ? f : -1);
        if (o < M::out_dim(net, i) && col >= 0) e = M::param_w_off(net, i) + o * in_full + col;
      }
    });
  });
  return e;
}

// Deterministic cross-workgroup reduction of the gradient slabs: a block owns 64
// consecutive slab offsets (coalesced reads) x 4 groups of slabs, each summed in
// slab order, then combined in a fixed order; the result is scattered to torch order.
template <class M>
__device__ __forceinline__ void grad_finalize_body(const float* __restrict__ slab, int ngrid, float* __restrict__ dparams,
                                                   int blk, float (*part)[64]) {
  const int lo = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int off = blk * 64 + lo;
  float v = 0.f;
  if (off < M::SLAB_TOTAL) {
    const int per = (ngrid + 3) / 4, g0 = grp * per, g1 = min(ngrid, g0 + per);
    const float* p = slab + off;
#pragma unroll 8
    for (int gi = g0; gi < g1; ++gi) v += p[(size_t)gi * M::SLAB_STRIDE];
  }
  part[grp][lo] = v;
  __syncthreads();
  if (grp == 0 && off < M::SLAB_TOTAL) {
    const int e = slab_to_param<M>(off);
    if (e >= 0) dparams[e] = (part[0][lo] + part[1][lo]) + (part[2][lo] + part[3][lo]);
  }
}
template <class M>
__global__ __launch_bounds__(256) void ude_grad_finalize_kernel(const float* __restrict__ slab, int ngrid,
                                                                float* __restrict__ dparams) {
  __shared__ float part[4][64];
  grad_finalize_body<M>(slab, ngrid, dparams, blockIdx.x, part);
}

// BAYES: the eps stream ([eval][N_PARAMS], torch order) re-laid out per evaluation in
// slab order (dW tiles in MFMA C order, bias rows), the layout the backward weights
// each evaluation's dW / bias sums with.  Padding slots get 0.
template <class M>
__global__ __launch_bounds__(256) void ude_eps_slab_kernel(const float* __restrict__ eps,
                                                           float* __restrict__ eslab) {
  const int off = blockIdx.x * 256 + threadIdx.x;
  const size_t ev = blockIdx.y;
  if (off >= M::SLAB_TOTAL) return;
  const int p = slab_to_param<M>(off);
  eslab[ev * M::SLAB_TOTAL + off] = p >= 0 ? eps[ev * M::N_PARAMS + p] : 0.f;
}

// ============================================================================
// Static-feature gradients (latent dims >= 3 are per-trajectory constants):
//   dW0[o][static s] = sum_n G0[n][o] * y0[n][static s]
//   dy0[n][static s] = sum_o W0[o][static s] * G0[n][o] + sum_j dlatent[j][n][static s]
// with G0[n][o] = sum over every evaluation of the layer-0 output gradient.
// ============================================================================
// dW0[:, static] split-K partials on MFMA: part[chunk][K0][S16] = sum over the
// chunk's tiles of G0[tile] (K0 x 16 trajectories) x X_static[tile] (16 x S16).
// Grid (STATIC_CHUNKS, STATIC_GROUPS): wave w of column group y owns static column tile
// 4y + w (every wave of the chip busy: the K0 x S16 x N GEMM is MFMA-issue bound);
// MFMA q covers trajectories 4g + q.  Tiles are walked two at a time so the next tile's
// operand loads are in flight during this tile's MFMAs.
template <class M>
__global__ __launch_bounds__(256) void ude_static_partial_kernel(const float* __restrict__ g0buf,
                                                                 const float* __restrict__ y0, int n_traj,
                                                                 int n_tiles, float* __restrict__ part) {
  constexpr int NOT = M::K0 / 16, NST = M::S16 / 16;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, t = lane & 15, g = lane >> 4;
  const int st = blockIdx.y * 4 + w;
  if (st >= NST) return;                             // no barriers or LDS in this kernel
  const int chunk = blockIdx.x;
  const int per = (n_tiles + M::STATIC_CHUNKS - 1) / M::STATIC_CHUNKS;
  const int tb = chunk * per, te = min(n_tiles, tb + per);
  const int s = st * 16 + t;
  const int r = s / (M::L - 3), cc = s - r * (M::L - 3);
  const bool s_ok = s < M::S;
  f4 acc[NOT];
#pragma unroll
  for (int o = 0; o < NOT; ++o) acc[o] = f4zero();
  #pragma unroll 2
  for (int tile = tb; tile < te; ++tile) {
    f4 a[NOT];
#pragma unroll
    for (int o = 0; o < NOT; ++o)
      a[o] = *reinterpret_cast<const f4*>(g0buf + ((size_t)tile * M::K0 + o * 16 + t) * TT + 4 * g);
    float b[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n = tile * TT + 4 * g + q;
      b[q] = (s_ok && n < n_traj) ? y0[((size_t)n * M::R + r) * M::L + 3 + cc] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int o = 0; o < NOT; ++o) acc[o] = mfma4(a[o][q], b[q], acc[o]);
  }
#pragma unroll
  for (int o = 0; o < NOT; ++o)
#pragma unroll
    for (int e = 0; e < 4; ++e)
      part[((size_t)chunk * M::K0 + o * 16 + 4 * g + e) * M::S16 + st * 16 + t] = acc[o][e];
}

template <class M>
__global__ __launch_bounds__(256) void ude_static_reduce_kernel(const float* __restrict__ part,
                                                                float* __restrict__ dparams) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= M::K0 * M::S) return;
  const int om = e / M::S, s = e - om * M::S;
  int net = 0, o = om;
  if (!M::HAS_P || om >= (M::HAS_P ? M::kout(0, 0) : 0)) {
    net = 1;
    o = om - (M::HAS_P ? M::kout(0, 0) : 0);
  }
  const int out = net == 0 ? M::out_dim(0, 0) : M::out_dim(1, 0);
  if (o >= out) return;
  float v = 0.f;
  for (int c = 0; c < M::STATIC_CHUNKS; ++c) v += part[((size_t)c * M::K0 + om) * M::S16 + s];
  const int w0 = net == 0 ? M::param_w_off(0, 0) : M::param_w_off(1, 0);
  dparams[w0 + (size_t)o * M::R * M::L + static_col<M>(s)] = v;
}

// d y0[:, static] = G0[tile]^T (16 x K0) x W0SP (K0 x S16) on MFMA, plus the direct
// cotangents of every output time (static latent dims are carried unchanged).
// One workgroup per trajectory tile; wave w owns static column tiles w, w + 4, ...
// The time sums read the tile's contiguous (16, R, L) block of every output time
// (coalesced, all dims) into LDS first: the static dims alone are a 5-of-8 stride.
template <class M>
__device__ __forceinline__ void dy0_static_body(const float* __restrict__ g0buf, const float* __restrict__ pack,
                                                const float* __restrict__ dlatent, int n_traj, int n_times,
                                                float* __restrict__ dy0, int tile, float* tsum) {
  // tsum: [TT][R][L] time sums of d latent (LDS)
  constexpr int NST = M::S16 / 16, SPW = (NST + 3) / 4, BLK = TT * M::R * M::L;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, t = lane & 15, g = lane >> 4;
  const size_t NRL = (size_t)n_traj * M::R * M::L;
  if (!dlatent) {                                    // static cotangents all zero
    #pragma unroll 1
    for (int i = threadIdx.x; i < BLK; i += 256) tsum[i] = 0.f;
  } else {
    const int nvalid = min(TT, n_traj - tile * TT) * M::R * M::L;
    const float* blk = dlatent + (size_t)tile * BLK;
    if constexpr ((M::R * M::L) % 4 == 0) {
      // 16-B loads, 8 output times in flight per lane (the sums stay in time order)
      #pragma unroll 1
      for (int i = 4 * threadIdx.x; i < BLK; i += 4 * 256) {
        f4 v = f4zero();
        if (i < nvalid) {
#pragma unroll 8
          for (int jt = 0; jt < n_times; ++jt) v += *reinterpret_cast<const f4*>(blk + (size_t)jt * NRL + i);
        }
        *reinterpret_cast<f4*>(tsum + i) = v;
      }
    } else {
      #pragma unroll 1
      for (int i = threadIdx.x; i < BLK; i += 256) {
        float v = 0.f;
        if (i < nvalid) {
#pragma unroll 8
          for (int jt = 0; jt < n_times; ++jt) v += blk[(size_t)jt * NRL + i];
        }
        tsum[i] = v;
      }
    }
  }
  __syncthreads();
  const float* gb = g0buf + (size_t)tile * M::K0 * TT;
  const float* wp = pack + M::W0SP_OFF;
  // operands in batches of QB k-steps, loaded unconditionally (column tiles past NST clamp
  // to the last one; their results are never stored) so a batch's loads are all in flight
  // before its MFMAs -- a guarded load per MFMA serialises on its latency
  constexpr int KQ = M::K0 / 4, QB = 8;
  int col[SPW];
#pragma unroll
  for (int j = 0; j < SPW; ++j) col[j] = min(w + 4 * j, NST - 1) * 16 + t;
  f4 acc[SPW];
#pragma unroll
  for (int j = 0; j < SPW; ++j) acc[j] = f4zero();
#pragma unroll
  for (int q0 = 0; q0 < KQ; q0 += QB) {
    float a[QB], b[QB][SPW];
#pragma unroll
    for (int qq = 0; qq < QB; ++qq) {
      if (q0 + qq < KQ) {
        const int k = 4 * (q0 + qq) + g;
        a[qq] = gb[k * TT + t];                        // A[traj t][o = k]
#pragma unroll
        for (int j = 0; j < SPW; ++j) b[qq][j] = wp[k * M::S16 + col[j]];
      }
    }
#pragma unroll
    for (int qq = 0; qq < QB; ++qq)
      if (q0 + qq < KQ)
#pragma unroll
        for (int j = 0; j < SPW; ++j) acc[j] = mfma4(a[qq], b[qq][j], acc[j]);
  }
#pragma unroll
  for (int j = 0; j < SPW; ++j) {
    const int s = (w + 4 * j) * 16 + t;
    if (w + 4 * j >= NST || s >= M::S) continue;
    const int r = s / (M::L - 3), cc = s - r * (M::L - 3);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int n = tile * TT + 4 * g + e;
      if (n < n_traj)
        dy0[((size_t)n * M::R + r) * M::L + 3 + cc] = acc[j][e] + tsum[((4 * g + e) * M::R + r) * M::L + 3 + cc];
    }
  }
}
template <class M>
__global__ __launch_bounds__(256) void ude_dy0_static_kernel(const float* __restrict__ g0buf,
                                                             const float* __restrict__ pack,
                                                             const float* __restrict__ dlatent, int n_traj,
                                                             int n_times, float* __restrict__ dy0) {
  extern __shared__ float tsum[];
  dy0_static_body<M>(g0buf, pack, dlatent, n_traj, n_times, dy0, blockIdx.x, tsum);
}

// ---- the backward's tail in ONE launch ----------------------------------------
// Three independent jobs, one block role each, run side by side instead of four launches in series:
//   [0, TCH * NST)              static weight gradient dW0[:, static] = sum_n G0[n] x_static[n]^T:
//                               block (chunk c, static column tile st), 4 waves over the chunk's tiles,
//                               summed in LDS in wave order, the chunk partial written; the last chunk
//                               block of column tile st to arrive (ticket on ctl[1 + st], agent-scope
//                               release / acquire) sums the TCH partials in chunk order and scatters
//                               them to torch order -- no separate reduce launch, deterministic
//   [.., + ngf)                 the gradient slabs' fixed-order sum (grad_finalize_body; BAYES: both
//                               halves)
//   [.., + n_tiles)             dy0 static of one trajectory tile (dy0_static_body: HBM-bound time sums
//                               of d latent + G0^T W0SP on MFMA)
// The latency-bound chunk blocks are dispatched first (blocks start in index order), the bandwidth-bound
// dy0 blocks fill the chip behind them.  ctl[1 ..] are zero on entry and left zero.
// static-gradient chunks: fewer, longer chunks win -- the last block's fixed-order sum of the chunk
// partials (device-coherent loads) is the tail's long pole (state49 bwd + tail 1.719 / 1.686 / 1.692 ms
// at 32 / 16 / 8 chunks, 1.737 / 1.810 at 64 / 128: profiles/r05/ab_tch_*.txt)
constexpr int TCH = 16;
template <class M>
struct Tail {
  static constexpr int NST = M::S16 / 16, NOT = M::K0 / 16;
  static constexpr int N_SP = M::HOIST ? TCH * NST : 0;
  static constexpr int NGF = (M::SLAB_TOTAL + 63) / 64;
  static constexpr int N_GF = NGF * (M::BAYES ? 2 : 1);
  // dynamic LDS: the dy0 tile's time sums, or 3 waves' static-gradient partial tiles
  static constexpr int LDS = cmax(M::HOIST ? TT * M::R * M::L * 4 : 0, 3 * NOT * 256 * 4 + 16);
  static int blocks(int n_tiles) { return (M::HOIST ? n_tiles : 0) + N_SP + N_GF; }
  // chunk partials [NST][TCH][NOT][64 lanes][4] (MFMA C order) behind the G0 sums
  static constexpr int64_t part_floats() { return M::HOIST ? (int64_t)NST * TCH * NOT * 256 : 0; }
};

template <class M>
__device__ void static_grad_chunk(const float* __restrict__ g0buf, const float* __restrict__ y0, int n_traj,
                                  int n_tiles, float* __restrict__ part, unsigned int* ctl,
                                  float* __restrict__ dparams, int c, int st, float* lds) {
  constexpr int NOT = Tail<M>::NOT, NST = Tail<M>::NST;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, t = lane & 15, g = lane >> 4;
  const int per = (n_tiles + TCH - 1) / TCH;
  const int tb = c * per, te = min(n_tiles, tb + per);
  const int s = st * 16 + t;
  const int r = s / (M::L - 3), cc = s - r * (M::L - 3);
  const bool s_ok = s < M::S;
  f4 acc[NOT];
#pragma unroll
  for (int o = 0; o < NOT; ++o) acc[o] = f4zero();
  #pragma unroll 4
  for (int tile = tb + w; tile < te; tile += WAVES) {
    f4 a[NOT];
#pragma unroll
    for (int o = 0; o < NOT; ++o)
      a[o] = *reinterpret_cast<const f4*>(g0buf + ((size_t)tile * M::K0 + o * 16 + t) * TT + 4 * g);
    float b[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n = tile * TT + 4 * g + q;
      b[q] = (s_ok && n < n_traj) ? y0[((size_t)n * M::R + r) * M::L + 3 + cc] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int o = 0; o < NOT; ++o) acc[o] = mfma4(a[o][q], b[q], acc[o]);
  }
  // the 4 waves' partial tiles summed in wave order (LDS), written as this chunk's partial
  f4* red = reinterpret_cast<f4*>(lds);
  if (w > 0) {
#pragma unroll
    for (int o = 0; o < NOT; ++o) red[((w - 1) * NOT + o) * 64 + lane] = acc[o];
  }
  __syncthreads();
  unsigned int* flag = reinterpret_cast<unsigned int*>(lds) + 3 * NOT * 256;   // behind the partial tiles
  if (w == 0) {
    // device-coherent (sc1) stores, acknowledged before the ticket (publish_fence; the ordering
    // argument and why no agent-scope fence: see finalize_stats_last)
    double* dst = reinterpret_cast<double*>(part + ((size_t)st * TCH + c) * NOT * 256);
#pragma unroll
    for (int o = 0; o < NOT; ++o) {
      const f4 v = ((acc[o] + red[o * 64 + lane]) + red[(NOT + o) * 64 + lane]) + red[(2 * NOT + o) * 64 + lane];
      __hip_atomic_store(dst + (o * 64 + lane) * 2, __builtin_bit_cast(double, __builtin_shufflevector(v, v, 0, 1)),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(dst + (o * 64 + lane) * 2 + 1, __builtin_bit_cast(double, __builtin_shufflevector(v, v, 2, 3)),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    publish_fence();
    unsigned int ticket = 0;
    if (lane == 0) ticket = __hip_atomic_fetch_add(ctl + 1 + st, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (lane == 0) *flag = ticket;
  }
  __syncthreads();
  if (*flag != TCH - 1) return;                      // block-uniform
  __asm__ __volatile__("" ::: "memory");             // the partial loads stay behind the ticket
  // last chunk of column tile st: the TCH partials in chunk order (device-coherent loads); element
  // (o, lane, e) is row o * 16 + 4 (lane / 16) + e, static column st * 16 + lane % 16
  const double* src = reinterpret_cast<const double*>(part + (size_t)st * TCH * NOT * 256);
  for (int i = threadIdx.x; i < NOT * 64; i += 256) {
    f4 v = f4zero();
    #pragma unroll 8
    for (int ch = 0; ch < TCH; ++ch) {
      const double* q = src + ((size_t)ch * NOT * 64 + i) * 2;
      typedef float f2 __attribute__((ext_vector_type(2)));
      const f2 lo = __builtin_bit_cast(f2, __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      const f2 hi = __builtin_bit_cast(f2, __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      const f4 u = {lo[0], lo[1], hi[0], hi[1]};
      v += u;
    }
    const int o = i >> 6, ln = i & 63;
    const int sc = st * 16 + (ln & 15);
    if (sc >= M::S) continue;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int om = o * 16 + 4 * (ln >> 4) + e;
      int net = 0, oo = om;
      if (!M::HAS_P || om >= (M::HAS_P ? M::kout(0, 0) : 0)) {
        net = 1;
        oo = om - (M::HAS_P ? M::kout(0, 0) : 0);
      }
      const int out = net == 0 ? M::out_dim(0, 0) : M::out_dim(1, 0);
      if (oo < out) {
        const int w0 = net == 0 ? M::param_w_off(0, 0) : M::param_w_off(1, 0);
        dparams[w0 + (size_t)oo * M::R * M::L + static_col<M>(sc)] = v[e];
      }
    }
  }
  if (threadIdx.x == 0) ctl[1 + st] = 0u;
  (void)NST;
}

template <class M>
__global__ __launch_bounds__(256) void ude_bwd_tail_kernel(const float* __restrict__ slab, int ngrid,
                                                           const float* __restrict__ g0buf,
                                                           const float* __restrict__ pack,
                                                           const float* __restrict__ y0,
                                                           const float* __restrict__ dlatent, int n_traj,
                                                           int n_tiles, int n_times, float* __restrict__ part,
                                                           unsigned int* ctl, float* __restrict__ dy0,
                                                           float* __restrict__ dparams) {
  extern __shared__ __attribute__((aligned(16))) float tl[];
  int b = blockIdx.x;
  if constexpr (M::HOIST) {
    if (b < Tail<M>::N_SP) {
      static_grad_chunk<M>(g0buf, y0, n_traj, n_tiles, part, ctl, dparams, b % TCH, b / TCH, tl);
      return;
    }
    b -= Tail<M>::N_SP;
  }
  if (b < Tail<M>::N_GF) {
    float (*pp)[64] = reinterpret_cast<float (*)[64]>(tl);
    if (M::BAYES && b >= Tail<M>::NGF)
      grad_finalize_body<M>(slab + M::SLAB_TOTAL, ngrid, dparams + M::N_PARAMS, b - Tail<M>::NGF, pp);
    else
      grad_finalize_body<M>(slab, ngrid, dparams, b, pp);
    return;
  }
  if constexpr (M::HOIST) dy0_static_body<M>(g0buf, pack, dlatent, n_traj, n_times, dy0, b - Tail<M>::N_GF, tl);
}

// fixed-order sum of per-workgroup fp64 partials -> one float (latent_init_loss of the DEC forward)
template <int V_ = 0>
__global__ void ude_sum_finalize_kernel(const double* __restrict__ part, int n, float* __restrict__ out) {
  const int ln = threadIdx.x;
  double s = 0.0;
  for (int i = ln; i < n; i += 64) s += part[i];
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m, 64);
  if (ln == 0) out[0] = (float)s;
}

template <int V_ = 0>
__global__ void ude_stats_finalize_kernel(double* __restrict__ slab, int ngrid, double n_eval,
                                          float* __restrict__ o_mean, float* __restrict__ o_std,
                                          float* __restrict__ o_norm) {
  // ... and the fp64 totals back into slab[0..4] (read by the data-parallel statistics exchange)
  // wave c sums statistic c: lane-strided partials, then a fixed butterfly (deterministic)
  __shared__ double tot[5];
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
  if (wv < 5) {
    double s = 0.0;
    for (int gi = ln; gi < ngrid; gi += 64) s += slab[(size_t)gi * 5 + wv];
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) s += __shfl_xor(s, m, 64);
    if (ln == 0) tot[wv] = s;
  }
  __syncthreads();
  const int c = threadIdx.x;
  if (c < 2) {
    const double m = tot[c] / n_eval;
    const double var = (tot[2 + c] - n_eval * m * m) / (n_eval - 1.0);
    if (o_mean) o_mean[c] = (float)m;
    if (o_std) o_std[c] = (float)sqrt(var > 0.0 ? var : 0.0);
  }
  if (c == 4 && o_norm) o_norm[0] = (float)sqrt(tot[4]);
  if (c < 5) slab[c] = tot[c];
}

}  // namespace ude
