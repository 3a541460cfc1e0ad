// Compile-time description of one UDE right-hand side (lib/models.py Fp / Fa / FaFp,
// lib/in_development/models_bayes.py Bayes_Fp / Bayes_Fa / Bayes_FaFp) and every
// derived layout the gfx950 kernels use.  All of it is constexpr so that per-wave
// register tiles (dW accumulators, static-hoist tiles) are indexed with compile-time
// constants and never spill to scratch.
//
// Reference layer rule (lib/models.py:118-124, :208-223, models_bayes.py:78-84): for
// hidden sizes [h1..hk] the Linears are in->h1, h1->h2, ..., hk->out with an ELU after
// Linear i only for i < k-1 (the last hidden Linear and the output Linear have no
// activation).  P-net ("net"/"Fp_net") outputs 2R rates, A-net ("aug_net") outputs 3R
// augmentation fluxes.
#pragma once

namespace ude {

constexpr int WAVES = 4;     // waves per workgroup (one per SIMD)
constexpr int TT = 16;       // trajectories per tile = the N of v_mfma_f32_16x16x4_f32
constexpr int NTHREADS = WAVES * 64;

constexpr int pad16(int x) { return (x + 15) & ~15; }
constexpr int cmax(int a, int b) { return a > b ? a : b; }
constexpr int cmin(int a, int b) { return a < b ? a : b; }

// KIND bit 4: Bayesian RHS (models_bayes.py Dense_Variational, :43-48): every
// evaluation uses its own weight sample w_e = mu + eps_e * |std|.
enum : int { KIND_FP = 1, KIND_FA = 2, KIND_FAFP = 3, KIND_BAYES = 4 };

template <int R_, int L_, int KIND_, int NPH_, int P0_, int P1_, int P2_, int P3_,
          int NAH_, int A0_, int A1_, int A2_, int A3_>
struct Model {
  static constexpr int R = R_, L = L_, KIND = KIND_;
  static constexpr bool HAS_P = (KIND & 1) != 0;
  static constexpr bool HAS_A = (KIND & 2) != 0;
  static constexpr bool BAYES = (KIND & KIND_BAYES) != 0;
  static constexpr int NPH = NPH_, NAH = NAH_;
  static constexpr int F = 3 * R;            // dynamic features: S, I, R of every region
  static constexpr int S = R * (L - 3);      // static features: latent dims >= 3 (zero derivative)
  static constexpr int F16 = pad16(F);
  static constexpr int S16 = pad16(S);
  // Deterministic weights: the static features' layer-0 contribution is a per-tile
  // constant (hoisted).  Bayesian weights change every evaluation, so layer 0 reads
  // [dynamic | static] features as one K = F16 + S16 input instead (FULL0).
  static constexpr bool HOIST = S > 0 && !BAYES;
  static constexpr bool FULL0 = S > 0 && BAYES;

  static constexpr int nl(int net) { return net == 0 ? (HAS_P ? NPH + 1 : 0) : (HAS_A ? NAH + 1 : 0); }
  static constexpr int D = cmax(nl(0), nl(1));
  static constexpr int nh(int net) { return net == 0 ? NPH : NAH; }
  static constexpr int hid(int net, int i) {
    return net == 0 ? (i == 0 ? P0_ : i == 1 ? P1_ : i == 2 ? P2_ : P3_)
                    : (i == 0 ? A0_ : i == 1 ? A1_ : i == 2 ? A2_ : A3_);
  }
  static constexpr bool has(int net, int i) { return i >= 0 && i < nl(net); }
  // layer-0 input width in the record: F dynamic features (FULL0: + the static ones
  // from F16 on, see col0)
  static constexpr int in_dim(int net, int i) { return i == 0 ? (FULL0 ? F16 + S : F) : hid(net, i - 1); }
  // layer-0 record feature f -> torch column of the flattened (R, L) state, -1 = padding
  static constexpr int col0(int f) {
    return f < F ? (f / 3) * L + (f % 3)
                 : (FULL0 && f >= F16 && f < F16 + S) ? ((f - F16) / (L - 3)) * L + 3 + (f - F16) % (L - 3) : -1;
  }
  static constexpr int out_dim(int net, int i) { return i < nh(net) ? hid(net, i) : (net == 0 ? 2 * R : 3 * R); }
  static constexpr bool act(int net, int i) { return i < nh(net) - 1; }
  static constexpr int kin(int net, int i) { return pad16(in_dim(net, i)); }
  static constexpr int kout(int net, int i) { return pad16(out_dim(net, i)); }
  static constexpr int rto(int net, int i) { return has(net, i) ? kout(net, i) / 16 : 0; }
  static constexpr int rti(int net, int i) { return has(net, i) ? kin(net, i) / 16 : 0; }
  static constexpr int K0 = (HAS_P ? kout(0, 0) : 0) + (HAS_A ? kout(1, 0) : 0);  // merged layer-0 rows

  // ---- forward row tiles at depth d: P tiles first, then A tiles -------------
  static constexpr int FT(int d) { return rto(0, d) + rto(1, d); }
  static constexpr int FTbase(int d) { int s = 0; for (int e = 0; e < d; ++e) s += FT(e); return s; }
  static constexpr int FTbase_total() { return FTbase(D); }
  static constexpr int fnet(int d, int k) { return k < rto(0, d) ? 0 : 1; }
  static constexpr int frt(int d, int k) { return k < rto(0, d) ? k : k - rto(0, d); }
  static constexpr int fowner(int d, int k) { return (FTbase(d) + k) % WAVES; }

  // ---- input-gradient (dX) row tiles at depth d --------------------------------
  // d > 0: rows are the inputs of layer d of each net; d == 0: the layer-0 input
  // features (both nets' layer-0 contributions summed in one accumulator).
  static constexpr int XT(int d) { return d == 0 ? (FULL0 ? F16 + S16 : F16) / 16 : rti(0, d) + rti(1, d); }
  static constexpr int xnet(int d, int m) { return m < rti(0, d) ? 0 : 1; }
  static constexpr int xrt(int d, int m) { return m < rti(0, d) ? m : m - rti(0, d); }
  static constexpr int xowner(int d, int m) {
    // start where the forward tiles of this depth stopped: spreads dW + dX work
    return (FTbase(d) + FT(d) + m) % WAVES;
  }

  // ---- per-wave register tiles -----------------------------------------------------
  static constexpr int ndw_before(int w, int d, int k) {
    int s = 0;
    for (int e = 0; e < D; ++e)
      for (int kk = 0; kk < FT(e); ++kk) {
        if (e == d && kk == k) return s;
        if (fowner(e, kk) == w) s += rti(fnet(e, kk), e);
      }
    return s;
  }
  static constexpr int NDW(int w) { return ndw_before(w, D, 0); }
  // dW tiles wave w accumulates in phase (layer) d
  static constexpr int ndw_phase(int w, int d) {
    int s = 0;
    for (int kk = 0; kk < FT(d); ++kk)
      if (fowner(d, kk) == w) s += rti(fnet(d, kk), d);
    return s;
  }
  static constexpr int max_ndw() { return cmax(cmax(NDW(0), NDW(1)), cmax(NDW(2), NDW(3))); }
  // BAYES keeps a second (eps-weighted) accumulator per dW tile in registers when both sets fit
  // and are small (the models_bayes.py class defaults, the R = 1 Fp / Fa nets).  Larger Bayesian
  // models (GST) store each evaluation's layer-output gradient rows instead and a separate kernel
  // (ude_gst_dw_kernel) forms every evaluation's weight gradient as one GEMM over the whole batch,
  // eps-weighting it there.  Above 12 dW tiles per wave GST wins even at R = 1: the US FaFp
  // [64,64,32]/[64,64] model (16) measured bwd 12.48 -> 10.33 ms, step 18.84 -> 17.16 ms on the
  // 4,096 x 365-step bayes_us workload (fwd 5.78 -> 6.13: it stores the stage inputs too;
  // tools/ab_gst_r1.py, profiles/r04/ab_gst_r1.log).
#ifndef UDE_GST_MIN_NDW
#define UDE_GST_MIN_NDW 12
#endif
  static constexpr bool GST = BAYES && max_ndw() > UDE_GST_MIN_NDW;
  static constexpr bool FITS = true;
  // ---- LDS record: one row of SR floats per trajectory ([t][feature]) ---------
  static constexpr int Y_OFF = 0;
  // FULL0: the static features sit right after the dynamic ones for the whole tile
  static constexpr int ACT0 = FULL0 ? F16 + S16 : F16;
  static constexpr int act_off(int net, int i) {
    int o = ACT0;
    for (int n = 0; n < 2; ++n)
      for (int j = 0; j < nl(n); ++j) {
        if (n == net && j == i) return o;
        o += kout(n, j);
      }
    return o;
  }
  static constexpr int ACT_END = act_off(2, 0);
  // static features in the record (HOIST: aliases the activation region, only live
  // outside the step loop; FULL0: persistent, right after the dynamic features)
  static constexpr int XSB_OFF = FULL0 ? F16 : F16 + K0;   // backward
  static constexpr int XSF_OFF = F16;                      // forward
  static constexpr int ALIAS_END = FULL0 ? ACT_END : cmax(ACT_END, F16 + K0 + S16);
  static constexpr int gbs(int net) {
    int m = 0;
    for (int j = 0; j < nl(net); ++j) m = cmax(m, kout(net, j));
    return m;
  }
  // GST (no weight gradients in the backward): the backward never reads the record's static features,
  // so the rate net's two gradient buffers live in their columns when they fit (R = 49: the record
  // then fits the LDS)
  static constexpr bool GB_IN_STATIC = GST && 2 * gbs(0) <= S16;
  static constexpr int gb_off(int net, int parity) {
    if (GB_IN_STATIC) return net == 0 ? F16 + parity * gbs(0) : ALIAS_END + parity * gbs(1);
    return ALIAS_END + (net == 0 ? 0 : 2 * gbs(0)) + parity * gbs(net);
  }
  static constexpr int gbuf(int net, int i) { return gb_off(net, i & 1); }
  // backward-only RK4 adjoint state, one [t][F] vector each (see bwd_body)
  // RK-state vectors are 12 * ceil(R/4) wide: the flux backward works on groups of
  // 4 regions (12 features) with 16-B LDS ops; QW = the matching width of the rates
  static constexpr int F4 = 12 * ((R + 3) / 4);
  static constexpr int SLOTS_ = (R * TT + NTHREADS - 1) / NTHREADS;   // == SLOTS
  static constexpr int QW = 8 * ((R + 3) / 4);
  // quads of the RK-state rows holding live features (3R of them; the rest stay zero): the
  // per-(trajectory, quad) RK passes of the backward touch only these
  static constexpr int NVL = (3 * R + 3) / 4;
  static constexpr int RK_A = ALIAS_END + (GB_IN_STATIC ? 0 : 2 * gbs(0)) + 2 * gbs(1);  // adjoint of y_{n+1}
  static constexpr int RK_PEND = RK_A + F4;       // y_n-side share of interpolated outputs
  static constexpr int RK_ACCY = RK_PEND + F4;    // adjoint of y_n being accumulated
  static constexpr int RK_DK1 = RK_ACCY + F4;
  static constexpr int RK_DK2 = RK_DK1 + F4;
  static constexpr int RK_DK3 = RK_DK2 + F4;
  // FULL0 backward: per-trajectory static-feature input gradients summed over the solve
  static constexpr int DYS_OFF = RK_DK3 + F4;
  // Small records (layer-0 input gradient split over the waves, SPLITX0; a rate net): the flux
  // part of each stage-input gradient is parked in its own row (DYF) and joined with the MLP part
  // before the ONE 3/8-rule adjoint update of the stage.  On trajectories whose infected share
  // grows exponentially the two parts nearly cancel; added to the fp32 adjoint accumulators one
  // after the other they cost ~20x the rounding of their sum (M1 Fp [32, 32]: dy0 5e-6 -> 3e-7
  // from the exact VJP of the same forward; found by oracle/ude_korder.c, tests/test_kernel_order.py).
  static constexpr bool DYF = HAS_P && (((F16 + (FULL0 ? S16 : 0)) / 16) < WAVES);
  static constexpr int DYF_OFF = DYS_OFF + (FULL0 ? S16 : 0);
  static constexpr int REC_F = cmax(ACT_END, F16 + S16);
  static constexpr int REC_B = DYF_OFF + (DYF ? F4 : 0);
  // row stride == 4 (mod 64) floats: conflict-free b128 fragment reads, and rows
  // t and t+4 land 16 banks apart for the dW b32 reads.
  static constexpr int stride(int n) { return ((n + 59) / 64) * 64 + 4; }
  static constexpr int SR_F = stride(REC_F);
  static constexpr int SR_B = stride(REC_B);
  static constexpr int LDS_F = TT * SR_F * 4;
  // + per-workgroup bias-gradient row sums (one float per forward row tile row)
  static constexpr int DB_LDS = TT * SR_B;
  static constexpr int NDB = 16 * FTbase_total();
  // BAYES: + the eps-weighted bias row sums (gradient of |b_std|)
  static constexpr int DBS_LDS = DB_LDS + NDB;
  // + staging slot for the next stage's checkpointed input ([t][F4], prefetched
  // during the flux pass)
  // (GST: no bias row sums, and the next stage's input is carried in registers: no staging slot)
  static constexpr int STG_LDS = DB_LDS + (GST ? 0 : (BAYES ? 2 : 1) * NDB);
  // SPLITX0: per-wave partial layer-0 input-gradient tiles [WAVES][XT(0)][64 lanes][4]
  static constexpr int X0P_LDS = STG_LDS + (GST ? 0 : TT * F4);
  // ---- stored activations (small models) ----------------------------------------------
  // At one tile per CU the backward's per-stage recompute of the forward (4 layer phases, each
  // a barrier-separated latency chain) costs more than streaming the activations through HBM:
  // the training forward writes each stage's activation rows [ACT0, ACT_END) of the record
  // ([tile][step][stage][16][ACT_A4], behind the stage checkpoint) and the backward stages them
  // back one stage ahead (ACT_STG) instead of recomputing.  288 GB of HBM makes this cheap:
  // 7.7 GB for the 4096 x 365-step north-star solve.
  static constexpr int ACT_A = ACT_END - ACT0;
  static constexpr int ACT_A4 = (ACT_A + 3) & ~3;
  static constexpr bool STORE_ACT = SLOTS_ == 1 && ACT_A4 <= 512;
  // Large records (R = 49: 162 KB of LDS, ~500 VGPRs in use) have no room to stage the next
  // stage's rows, so the backward loads each stage's rows straight into the record at the stage
  // start (STORE_ACT_D): one exposed HBM latency per stage instead of the recompute's four
  // barrier-separated layer phases (a third of the backward's MFMA work).  1.5 GB for the
  // 20,480-trajectory x 8-step state49 solve.
  static constexpr bool STORE_ACT_D = !STORE_ACT && (!BAYES || GST);
  static constexpr bool ACT_STORED = STORE_ACT || STORE_ACT_D;
  // Two waves per SIMD in the backward of small deterministic records (SPLIT_BWD): at one tile
  // per CU a single wave per SIMD leaves every LDS latency, epilogue and barrier of a stage's
  // critical path (flux -> input gradients layer by layer -> RK adjoint) exposed.  Waves 0-3
  // run that path; waves 4-7 accumulate the weight gradients of the same phase (which nothing
  // in the stage waits for) from the same LDS operands, on the same SIMDs, so their MFMAs fill
  // the critical path's gaps.  Not for Bayes: the partner waves would hold the plain and the
  // eps-weighted dW (2 x 128 VGPRs at [64,64,32]) and spill (measured M1 bwd 21.2 ms vs 12.4 ms for
  // the 4-wave kernel at one wave per SIMD).
  static constexpr bool SPLIT_BWD = STORE_ACT && SLOTS_ == 1 && !BAYES;
  // Large records (STORE_ACT_D) split the same way (SPLIT_BWD_L): waves 4-7 (bwd_wbody_l) hold the
  // weight-gradient accumulators (the ~176 VGPRs per wave that kept the 4-wave kernel at one wave per
  // SIMD) and move the next stage's data with LDS-DMA (global_load_lds): each layer's activation rows
  // once the current stage's last reader of that layer is past its barrier (issued behind the next
  // phase's MFMAs), and the checkpointed stage input into the staging slot -- no data registers, no
  // exposed load at the stage start.
#ifndef UDE_NO_SPLIT_L
  static constexpr bool SPLIT_BWD_L = STORE_ACT_D && !BAYES;
#else
  static constexpr bool SPLIT_BWD_L = false;
#endif
  static constexpr bool SPLITB = SPLIT_BWD || SPLIT_BWD_L;
  // Backward critical path with weights read from L2 (GST; SPLIT_BWD_L's waves 0-3; every Bayesian
  // backward, whose per-evaluation samples are never register-resident): each phase's input-gradient
  // fragments are loaded one phase ahead (the first phase's before the flux pass), so no phase waits
  // on the L2 latency (Bayes M1 bwd 13.4 -> 12.4 ms)
  static constexpr bool PF_X = GST || SPLIT_BWD_L || BAYES;
  static constexpr int BWD_THREADS = SPLITB ? 2 * NTHREADS : NTHREADS;
  // Training forward of small records at one tile per CU: four more waves copy each stage's
  // activation rows from the record to HBM during the flux pass, off the critical path
  // (ude_kernels.h fwd_sbody).  With more tiles than CUs two 4-wave workgroups per CU win.
  static constexpr bool SPLIT_FWD = STORE_ACT && SLOTS_ == 1 && !GST;
  // Stored row layout ([tile][step][stage][16][XST_W] behind the checkpoint): the activation rows
  // [ACT0, ACT_END) of the record at column ACT_IN.  GST rows also carry the stage input [0, F16)
  // in front (written by the flux pass before it overwrites the Y slot): the weight-gradient GEMM
  // multiplies the layer-0 output gradients by [stage input | static features] per evaluation.
  static constexpr int ACT_IN = GST ? F16 : 0;
  static constexpr int XST_W = ACT_IN + ACT_A4;
  static constexpr int ACT_STG = X0P_LDS + (XT(0) < WAVES ? WAVES * XT(0) * 256 : 0);
  static constexpr int LDS_B = (ACT_STG + (STORE_ACT ? TT * ACT_A4 : 0)) * 4;
  static_assert(LDS_F <= 160 * 1024 && LDS_B <= 160 * 1024, "record does not fit the 160 KiB LDS");

  // ---- packed weights (fragment order, 16-B per lane per MFMA quad) --------------
  //  WF(net,i): [rto][kin/16][64 lanes][4]   A operand of the forward GEMM
  //  WT(net,i): [rti][kout/16][64][4]        A operand of the input-gradient GEMM
  //  B(net,i):  [kout]                       bias, zero padded
  //  WSF(net):  [rto(net,0)][S16/16][64][4]  layer-0 static columns (per-tile hoist)
  //  W0SP:      [K0][S16]                    layer-0 static columns, plain, merged nets (dy0 static)
  // BAYES: one such pack per RHS evaluation (PACK_TOTAL floats apart), no WSF / W0SP.
  static constexpr int wf_size(int net, int i) { return has(net, i) ? rto(net, i) * (kin(net, i) / 16) * 256 : 0; }
  static constexpr int wt_size(int net, int i) { return has(net, i) ? rti(net, i) * (kout(net, i) / 16) * 256 : 0; }
  static constexpr int b_size(int net, int i) { return has(net, i) ? kout(net, i) : 0; }
  static constexpr int layer_pack_size(int net, int i) { return wf_size(net, i) + wt_size(net, i) + b_size(net, i); }
  static constexpr int layer_pack_off(int net, int i) {
    int o = 0;
    for (int n = 0; n < 2; ++n)
      for (int j = 0; j < nl(n); ++j) {
        if (n == net && j == i) return o;
        o += layer_pack_size(n, j);
      }
    return o;
  }
  static constexpr int wf_off(int net, int i) { return layer_pack_off(net, i); }
  static constexpr int wt_off(int net, int i) { return layer_pack_off(net, i) + wf_size(net, i); }
  static constexpr int b_off(int net, int i) { return wt_off(net, i) + wt_size(net, i); }
  static constexpr int LAYERS_END = layer_pack_off(2, 0);
  static constexpr int wsf_size(int net) { return (HOIST && has(net, 0)) ? rto(net, 0) * (S16 / 16) * 256 : 0; }
  static constexpr int wsf_off(int net) { return LAYERS_END + (net == 0 ? 0 : wsf_size(0)); }
  static constexpr int W0SP_OFF = LAYERS_END + wsf_size(0) + wsf_size(1);
  static constexpr int W0SP_SIZE = HOIST ? K0 * S16 : 0;
  static constexpr int PACK_TOTAL = W0SP_OFF + W0SP_SIZE;

  // ---- per-workgroup gradient slab -------------------------------------------------
  static constexpr int dyn_tiles_before(int d, int k) {
    int s = 0;
    for (int e = 0; e < D; ++e)
      for (int kk = 0; kk < FT(e); ++kk) {
        if (e == d && kk == k) return s;
        s += rti(fnet(e, kk), e);
      }
    return s;
  }
  static constexpr int N_DYN_TILES = dyn_tiles_before(D, 0);
  static constexpr int NCS = S16 / 16;
  static constexpr int SLAB_DB = N_DYN_TILES * 256;
  static constexpr int SLAB_TOTAL = SLAB_DB + FTbase(D) * 16;
  // BAYES: each workgroup slab holds [d mean | d |std|]; the eps stream is laid out
  // per evaluation in this same slab order (SLAB_TOTAL floats per evaluation)
  static constexpr int SLAB_STRIDE = SLAB_TOTAL * (BAYES ? 2 : 1);
  // static-feature gradient work (outside the main kernel, HOIST only): per-tile
  // layer-0 row sums G0[tile][K0][16] and split-K partials of dW0[:, static]
  static constexpr int STATIC_CHUNKS = 128;
  static constexpr int STATIC_GROUPS = (S16 / 16 + 3) / 4;

  static constexpr int ng_before(int w, int d, int k) {
    int s = 0;
    for (int e = 0; e < D; ++e)
      for (int kk = 0; kk < FT(e); ++kk) {
        if (e == d && kk == k) return s;
        if (fowner(e, kk) == w) s += 1;
      }
    return s;
  }
  static constexpr int NG(int w) { return ng_before(w, D, 0); }
  static constexpr int own_phase(int w, int d) {
    int s = 0;
    for (int k = 0; k < FT(d); ++k) if (fowner(d, k) == w) s += 1;
    return s;
  }
  // input-gradient tiles wave w owns in phase d; its first owned forward tile of phase d (0 if none)
  static constexpr int own_x(int w, int d) {
    int s = 0;
    for (int m = 0; m < XT(d); ++m) if (xowner(d, m) == w) s += 1;
    return s;
  }
  static constexpr int first_owned(int w, int d) {
    for (int k = 0; k < FT(d); ++k) if (fowner(d, k) == w) return k;
    return 0;
  }
  static constexpr int nz_before(int w, int k) {
    int s = 0;
    for (int kk = 0; kk < k; ++kk) if (fowner(0, kk) == w) s += 1;
    return s;
  }
  static constexpr int NZ(int w) { return nz_before(w, FT(0)); }

  // weight-fragment quads (16-B per lane) a wave prefetches per phase
  static constexpr int fq_before(int w, int d, int k) {
    int s = 0;
    for (int kk = 0; kk < k; ++kk) if (fowner(d, kk) == w) s += kin(fnet(d, kk), d) / 16;
    return s;
  }
  static constexpr int FQ(int w, int d) { return fq_before(w, d, FT(d)); }
  static constexpr bool owns_f(int w, int d, int net) {
    for (int k = 0; k < FT(d); ++k) if (fowner(d, k) == w && fnet(d, k) == net) return true;
    return false;
  }
  static constexpr bool owns_x(int w, int d, int net) {
    for (int m = 0; m < XT(d); ++m) if (xowner(d, m) == w && (d == 0 || xnet(d, m) == net)) return true;
    return false;
  }
  static constexpr int xq(int d, int m) {
    return d == 0 ? (HAS_P ? kout(0, 0) / 16 : 0) + (HAS_A ? kout(1, 0) / 16 : 0) : kout(xnet(d, m), d) / 16;
  }
  // Layer-0 input gradient with fewer feature tiles than waves (small R): instead of one
  // wave running a tile's whole K = K0 chain, every wave takes the K quads qq = w (mod 4) of
  // every tile and the 4 partial tiles are summed afterwards (bwd_body, fixed order).
  static constexpr int X0Q = (HAS_P ? kout(0, 0) / 16 : 0) + (HAS_A ? kout(1, 0) / 16 : 0);
  static constexpr bool SPLITX0 = XT(0) < WAVES;
  static constexpr int x0q_w(int w) { int s = 0; for (int qq = 0; qq < X0Q; ++qq) if (qq % WAVES == w) s += 1; return s; }
  static constexpr int xq_before(int w, int d, int m) {
    if (d == 0 && SPLITX0) return m * x0q_w(w);
    int s = 0;
    for (int mm = 0; mm < m; ++mm) if (xowner(d, mm) == w) s += xq(d, mm);
    return s;
  }
  static constexpr int XQ(int w, int d) { return xq_before(w, d, XT(d)); }

  // ---- register-resident weights (small models) ---------------------------------
  // A wave's weight fragments never change during a launch (deterministic RHS): when all
  // of them fit next to the working set they are loaded once into VGPRs instead of being
  // re-read from L2 at every layer phase (at R = 1 that L2 latency, not the MFMA work,
  // paced every phase).  Per wave: forward fragments, bias quads, input-gradient fragments.
  static constexpr bool has_bias(int d) { return !(d == 0 && HOIST); }
  static constexpr int nb_phase(int w, int d) {
    int s = 0;
    if (has_bias(d))
      for (int k = 0; k < FT(d); ++k) if (fowner(d, k) == w) s += 1;
    return s;
  }
  static constexpr int nb_before(int w, int d, int k) {
    int s = 0;
    if (has_bias(d))
      for (int kk = 0; kk < k; ++kk) if (fowner(d, kk) == w) s += 1;
    return s;
  }
  static constexpr int fq_base(int w, int d) { int s = 0; for (int e = 0; e < d; ++e) s += FQ(w, e); return s; }
  static constexpr int nb_base(int w, int d) { int s = 0; for (int e = 0; e < d; ++e) s += nb_phase(w, e); return s; }
  static constexpr int xq_base(int w, int d) { int s = 0; for (int e = 0; e < d; ++e) s += XQ(w, e); return s; }
  static constexpr int WF_Q(int w) { return fq_base(w, D); }
  static constexpr int WB_Q(int w) { return nb_base(w, D); }
  static constexpr int WX_Q(int w) { return xq_base(w, D); }
  static constexpr int wreg_q(int w) { return WF_Q(w) + WB_Q(w) + WX_Q(w); }
  static constexpr int max_wreg_q() { return cmax(cmax(wreg_q(0), wreg_q(1)), cmax(wreg_q(2), wreg_q(3))); }
  static constexpr int WREG_MAX_Q = 56;      // <= 224 VGPRs of resident fragments per wave
  static constexpr bool WREG = !BAYES && max_wreg_q() <= WREG_MAX_Q;
  // forward-only resident fragments at one workgroup per CU (ude_fwd_kernel RES): <= 96 quads
  static constexpr int fwd_wreg_q(int w) { return WF_Q(w) + WB_Q(w); }
  static constexpr bool FWD_RES = !BAYES && !WREG &&
                                  cmax(cmax(fwd_wreg_q(0), fwd_wreg_q(1)), cmax(fwd_wreg_q(2), fwd_wreg_q(3))) <= 96;
  // Bayesian forward with few fragments per wave: each evaluation's sample in registers, prefetched
  // during the previous evaluation's flux pass (fwd_body PFB)
  static constexpr bool FWD_PFB = BAYES &&
                                  cmax(cmax(fwd_wreg_q(0), fwd_wreg_q(1)), cmax(fwd_wreg_q(2), fwd_wreg_q(3))) <= 40;

  // ---- parameters in torch order (nn.Linear weight (out,in) then bias) ----------------
  static constexpr int param_w_off(int net, int i) {
    int o = 0;
    for (int n = 0; n < 2; ++n)
      for (int j = 0; j < nl(n); ++j) {
        if (n == net && j == i) return o;
        o += out_dim(n, j) * (j == 0 ? R * L : in_dim(n, j)) + out_dim(n, j);
      }
    return o;
  }
  static constexpr int N_PARAMS = param_w_off(2, 0);
  // floats of the flat gradient output: BAYES = [d mean (torch order) | d |std|]
  static constexpr int N_GRAD = N_PARAMS * (BAYES ? 2 : 1);
  static constexpr int PAIRS = R * TT;
  static constexpr int SLOTS = (PAIRS + NTHREADS - 1) / NTHREADS;

  // ---- decoder epilogue (lib/models.py:27-51 Decoder = Linear(3R -> R) on
  // latent[..., :3], lib/VAE.py:138) ------------------------------------------------------
  // The training forward can emit y_hat = W_dec . y[:3R] + b_dec at every output time instead of
  // the (T, N, R, L) latent: one more small GEMM out[o][t] = W_dec[o][:] . Y[t][:] over the
  // record's Y slot (its 3R features are exactly the decoder's flattened (R, 3) input order).
  // Packed like a forward layer: [RTD][F16/16][64 lanes][4] fragments, then the bias [RTD * 16].
  static constexpr int RTD = pad16(R) / 16;
  static constexpr int DEC_WF = RTD * (F16 / 16) * 256;
  static constexpr int DEC_PACK = DEC_WF + RTD * 16;
  // DEC forward: per-thread fp64 latent_init_loss partials behind the forward record
  static constexpr int REG_LDS_F = TT * SR_F;
  static constexpr int LDS_F_DEC = LDS_F + NTHREADS * 8;
};

// The same model without stored activations (memory fallback, UdeProblem.recompute): the training
// forward stores only the 3R stage inputs per stage and the backward re-runs each stage's layer
// phases from them (long-horizon row) -- O(steps * 3R) floats per trajectory instead of
// O(steps * activations).  Every kernel reads these through M::, so the derived names win.
template <class B>
struct Recompute : B {
  static constexpr bool STORE_ACT = false, STORE_ACT_D = false, ACT_STORED = false;
  static constexpr bool SPLIT_BWD = false, SPLIT_FWD = false, SPLIT_BWD_L = false, SPLITB = false;
  static constexpr int BWD_THREADS = NTHREADS;
  static constexpr int LDS_B = B::ACT_STG * 4;
  static constexpr int LDS_F_DEC = B::LDS_F + NTHREADS * 8;
};

}  // namespace ude
