// Fused per-point viscoelastic update (Narayanaswamy shift, partial fictive
// temperatures, strains, scaled time, Prony-series stress increments), gfx950.
//
// Replaces the 17 dolfinx fem::interpolate(Expression) passes of one time step
// (ThermoViscoProblem.py:393-595) over the FFCx expression kernels of
// ViscoelasticModel._init_expressions (ViscoelasticModel.py:86-242), together
// with the _update_values copies (ThermoViscoProblem.py:349-354) and the final
// T_prev <- T update (ThermoViscoProblem.py:378-379).
//
// For degree-1 Lagrange spaces every expression is a per-dof map, so one thread
// owns one dof and carries the whole pipeline in registers: a single HBM pass
// that reads T, T_prev, Tf_partial and writes the state (Tf_partial, Tf, phi,
// xi, sigma) — plus every intermediate Function of the reference when
// materialize = all.  s_tilde / sigma_tilde (Q3: fed only by themselves, so
// +0.0 from the zero initial state on) are read and rewritten only once a
// value other than +0.0 has appeared (ViscoFields::tflag); until then they
// cost no HBM traffic.
//
// Semantics follow the reference, quirks included:
//   Q1 phi is Eq. 5 (the Eq. 25 expression is overwritten, VEM:100 vs :156);
//   Q2 Tf_prev is overwritten before the thermal strain reads it (TVP:481 vs
//      :492), so the alpha_liquid term is (Tf - Tf) = 0;
//   Q3 s_tilde / sigma_tilde are fed by their own previous values (VEM:196,205);
//   Q4 xi = dt/2 (phi_next - phi) with "-" (VEM:171);
//   Q5 xi == 0 gives 0/0 = NaN in ds / dsigma (VEM:178,187).
// The arithmetic is written in the reference's operator order and this file is
// compiled with -ffp-contract=off, so it performs the same IEEE operations as
// the CPU oracle (exp() may differ by an ulp between libm and ocml).
//
// Layout: component-major (SoA) fields, comp * stride + dof, so every load and
// store of a wavefront is one contiguous 512-byte segment.
#include "tv_internal.h"

namespace tv {
namespace {

__device__ __forceinline__ double taylor_E(double xi, double lam) {
  // ViscoelasticModel._taylor_exponential: sum_{k=0}^{2} 1/k! (-xi/lam)^k,
  // summed left to right (np.sum over a Python list).
  const double x = (-xi) / lam;
  const double t0 = 1.0;          // 1/0! * x**0 (== 1 also for NaN/inf x)
  const double t1 = 1.0 * x;      // 1/1! * x**1
  const double t2 = 0.5 * (x * x);  // 1/2! * x**2
  return (t0 + t1) + t2;
}

struct TState {
  double T, Tp, Tf, Tfo, xi;  // Tfo: Tf of the previous step (paper mode's strain)
};

// T-family part: phi, Tf_partial, Tf, T_next, phi_next, xi at T-dof t.
// PAPER (opt-in model_mode, never the default): Eq. 25 drives Eq. 24, the
// thermal strain sees Tf - Tf_prev of the previous step, and xi takes the
// trapezoidal "+" (the fixes of SURVEY.md A.3 Q1, Q2, Q4).
template <bool ALL, bool PAPER>
__device__ __forceinline__ TState t_part(const ViscoConst& c, const ViscoFields& f, int64_t t) {
  TState o;
  const double T = f.T[t];
  const double Tp = f.Tp[t];
  const double Tfo = PAPER ? f.Tf[t] : 0.0;
  // the six previous partial fictive temperatures loaded with T and T_prev,
  // before any store: loaded one by one, each load waited behind the store
  // before it (the compiler cannot prove that i sT + t and (i + 1) sT + t
  // differ) -- six memory round trips per dof
  double prev6[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) prev6[i] = f.Tfp[i * f.sT + t];
  // (without the fence the scheduler sinks each load to just before its first
  // use, between the divisions: one round trip per load again)
  __builtin_amdgcn_sched_barrier(0);
  // Eq. 5 (VEM:156-161)
  const double phi = exp(c.H_over_Rg * (c.inv_Tb - 1.0 / T));
  // Eq. 25 (VEM:100-108), overwritten by Eq. 5 in the reference (Q1)
  const double phi_tf = PAPER ? exp(c.H_over_Rg * ((c.inv_Tb - c.chi / T) - (1.0 - c.chi) / Tfo)) : phi;
  // Eq. 24 (VEM:111-119), Tf_partial_prev -> Tf_partial (alias: TVP:469-470)
  double Tf = 0.0;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const double prev = prev6[i];
    const double cur = (c.lambda_m[i] * prev + T * c.dt * phi_tf) / (c.lambda_m[i] + c.dt * phi_tf);
    f.Tfp[i * f.sT + t] = cur;
    Tf = Tf + c.m_n[i] * cur;  // Eq. 26 inner(m, Tf_partial) (VEM:122-125)
  }
  f.Tf[t] = Tf;  // Tf_prev <- Tf (alias: TVP:481-482; PAPER: the strain keeps Tfo)
  // extrapolation (VEM:150-153)
  const double Tn = T + (T - Tp);
  // phi again (identical, VEM:156) and phi_next (VEM:162-167)
  const double phin = exp(c.H_over_Rg * (c.inv_Tb - 1.0 / Tn));
  // Eq. 19 with "-" (VEM:170-173, Q4), PAPER: "+"
  const double xi = PAPER ? c.half_dt * (phin + phi) : c.half_dt * (phin - phi);
  f.phi[t] = phi;
  f.xi[t] = xi;
  if (ALL) {
    f.Tn[t] = Tn;
    f.phin[t] = phin;
  }
  o.T = T; o.Tp = Tp; o.Tf = Tf; o.Tfo = PAPER ? Tfo : Tf; o.xi = xi;
  return o;
}

// The total stress (9 write-only streams, a third of the update's HBM bytes) is
// stored non-temporally: 409 -> 355 us at C4 (measured); the read-modify-write
// Tf_partial streams stored that way measured slower.
// sigma-family part at sigma-dof s given the T-family values of its source dof.
// LEAN: s_tilde / sigma_tilde are known to be +0.0 everywhere (f.tflag == 0);
// the products 0 * E are formed exactly as in the reference (one value per
// Prony term: the same for all d*d components), but stored only when one of
// them is not +0.0 (E not finite, e.g. xi = NaN) -- a single rare branch per
// dof -- which also raises `dirty` so the next launches read the fields
// again.  Memory therefore always holds the exact values, in both modes.
// PAPER: Eq. 16 feeds s~ / sigma~ from the previous s / sigma partial stresses
// (Q3 fixed), which are then state fields (never LEAN).
template <int D, bool ALL, bool LEAN, bool PAPER = false>
__device__ __forceinline__ void s_part(const ViscoConst& c, const ViscoFields& f, int64_t s, const TState& ts,
                                       bool& dirty) {
  constexpr int DD = D * D;
  static_assert(!(LEAN && PAPER), "paper mode carries s / sigma partial state");
  // Eq. 9 (VEM:128-133): I*(alpha_s (T - T_prev) + (alpha_l - alpha_s)(Tf - Tf_prev)), Tf_prev == Tf (Q2)
  const double scal = c.alpha_s * (ts.T - ts.Tp) + c.dalpha * (ts.Tf - ts.Tfo);
  double tot[DD];
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const double th = (i == j ? 1.0 : 0.0) * scal;
      tot[i * D + j] = -th;  // Eq. 28 (VEM:136-139)
      if (ALL) {
        f.th[(i * D + j) * f.sS + s] = th;
        f.tot[(i * D + j) * f.sS + s] = -th;
      }
    }
  double tr = 0.0;
#pragma unroll
  for (int i = 0; i < D; ++i) tr = tr + tot[i * D + i];
  double dev[DD];
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int j = 0; j < D; ++j) {
      // Eq. 29 (VEM:142-146): eps - 1/dim * I * tr(eps)
      dev[i * D + j] = tot[i * D + j] - (c.inv_dim * (i == j ? 1.0 : 0.0)) * tr;
      if (ALL) f.dev[(i * D + j) * f.sS + s] = dev[i * D + j];
    }
  const double xi = ts.xi;
  double sig[DD];
  uint64_t tz = 0;  // LEAN: bits of every 0 * E product
  auto term = [&](const int n) {
    const double Eg = taylor_E(xi, c.lambda_g[n]);
    const double Ek = taylor_E(xi, c.lambda_k[n]);
    const double twog = 2.0 * c.g_n[n];
    const double omEg = 1.0 - Eg, omEk = 1.0 - Ek;
#pragma unroll
    for (int q = 0; q < DD; ++q) {
      const int i = q / D, j = q % D;
      const int64_t o = (int64_t)(n * DD + q) * f.sS + s;
      // Eq. 15a + 20 (VEM:176-182)
      const double ds = (((twog * dev[q]) / xi) * c.lambda_g[n]) * omEg;
      // Eq. 16a (VEM:195-200)
      const double st = (LEAN ? 0.0 : (PAPER ? f.sp[o] : f.st[o])) * Eg;
      if (LEAN) tz |= (uint64_t)__double_as_longlong(st);
      // Eq. 17a (VEM:212-215)
      const double sp = ds + st;
      // Eq. 15b + 20 (VEM:185-191)
      const double dsg = (((c.k_n[n] * (tr * (i == j ? 1.0 : 0.0))) / xi) * c.lambda_k[n]) * omEk;
      // Eq. 16b (VEM:203-209)
      const double sgt = (LEAN ? 0.0 : (PAPER ? f.sgp[o] : f.sgt[o])) * Ek;
      if (LEAN) tz |= (uint64_t)__double_as_longlong(sgt);
      // Eq. 17b (VEM:218-221)
      const double sgp = dsg + sgt;
      if (!LEAN) {
        f.st[o] = st;    // next -> current copy (TVP:559-560)
        f.sgt[o] = sgt;  // (TVP:578-581)
      }
      if (ALL) {
        f.ds[o] = ds;
        f.dsig[o] = dsg;
      }
      if (ALL || PAPER) {
        f.sp[o] = sp;
        f.sgp[o] = sgp;
      }
      // Eq. 18 (VEM:224-228), np.sum over n left to right
      sig[q] = (n == 0) ? (sp + sgp) : sig[q] + (sp + sgp);
    }
    };
  if constexpr (LEAN) {  // no loads: the whole term chain unrolled
#pragma unroll
    for (int n = 0; n < 6; ++n) term(n);
  } else {  // 2 d*d tilde loads per term in flight, not 12 d*d (register budget)
#pragma unroll 1
    for (int n = 0; n < 6; ++n) term(n);
  }
#pragma unroll
  for (int q = 0; q < DD; ++q) __builtin_nontemporal_store(sig[q], &f.sigma[(int64_t)q * f.sS + s]);  // write-only stream
  if (LEAN && tz != 0) {  // a non-finite E: materialise this dof's tilde values
#pragma unroll 1
    for (int n = 0; n < 6; ++n) {
      const double st = 0.0 * taylor_E(xi, c.lambda_g[n]);
      const double sgt = 0.0 * taylor_E(xi, c.lambda_k[n]);
#pragma unroll 1
      for (int q = 0; q < DD; ++q) {
        const int64_t o = (int64_t)(n * DD + q) * f.sS + s;
        f.st[o] = st;
        f.sgt[o] = sgt;
      }
    }
    dirty = true;
  }
}

template <int D, bool ALL, bool LEAN, bool PAPER = false>
__device__ __forceinline__ void fused_loop(const ViscoConst& c, const ViscoFields& f) {
  bool dirty = false;
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < f.n; t += (int64_t)gridDim.x * kBlock) {
    const int64_t dT = f.off_T + t;
    const TState ts = t_part<ALL, PAPER>(c, f, dT);
    s_part<D, ALL, LEAN, PAPER>(c, f, f.off_S + t, ts, dirty);
    if (f.copy_Tprev) f.Tp[dT] = ts.T;  // TVP:378-379, T_prev is not read after this point
  }
  if (dirty) *f.tflag = 1;
}

template <int D, bool ALL>
__global__ __launch_bounds__(kBlock) void k_visco_fused(ViscoConst c, ViscoFields f) {
  if (!newton_gate_open(f.gate)) return;
  if (c.paper) {
    fused_loop<D, ALL, false, true>(c, f);
    return;
  }
  // read once: a flag raised later in this launch changes nothing (see s_part)
  if (*f.tflag == 0) fused_loop<D, ALL, true>(c, f);
  else fused_loop<D, ALL, false>(c, f);
}

// mixed families, T pass; in paper mode it also keeps the previous step's Tf
// per T dof (f.Tfo, a work array) for the sigma pass's thermal strain
template <bool ALL>
__global__ __launch_bounds__(kBlock) void k_visco_T(ViscoConst c, ViscoFields f) {
  if (!newton_gate_open(f.gate)) return;
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < f.n; t += (int64_t)gridDim.x * kBlock) {
    if (c.paper) {
      const TState ts = t_part<ALL, true>(c, f, f.off_T + t);
      f.Tfo[f.off_T + t] = ts.Tfo;
    } else {
      (void)t_part<ALL, false>(c, f, f.off_T + t);
    }
  }
}

// mixed families: sigma dof s reads the T-family values of the dof that the
// last cell written by fem::interpolate assigns to it (f.map).
template <int D, bool ALL, bool LEAN, bool PAPER = false>
__device__ __forceinline__ void s_loop(const ViscoConst& c, const ViscoFields& f) {
  bool dirty = false;
  for (int64_t s = blockIdx.x * (int64_t)kBlock + threadIdx.x; s < f.n; s += (int64_t)gridDim.x * kBlock) {
    const int64_t t = f.map[s];
    TState ts;
    ts.T = f.T[t];
    ts.Tp = f.Tp[t];
    ts.Tf = f.Tf[t];
    ts.Tfo = PAPER ? f.Tfo[t] : ts.Tf;
    ts.xi = f.xi[t];
    s_part<D, ALL, LEAN, PAPER>(c, f, f.off_S + s, ts, dirty);
  }
  if (dirty) *f.tflag = 1;
}

template <int D, bool ALL>
__global__ __launch_bounds__(kBlock) void k_visco_S(ViscoConst c, ViscoFields f) {
  if (!newton_gate_open(f.gate)) return;
  if (c.paper) s_loop<D, ALL, false, true>(c, f);
  else if (*f.tflag == 0) s_loop<D, ALL, true>(c, f);
  else s_loop<D, ALL, false>(c, f);
}

__global__ __launch_bounds__(kBlock) void k_copy_gated(double* __restrict__ d, const double* __restrict__ s, int64_t n,
                                                       NewtonGate g) {
  if (!newton_gate_open(g)) return;
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < n; t += (int64_t)gridDim.x * kBlock) d[t] = s[t];
}

int blocks_for(int64_t n) {
  int64_t b = (n + kBlock - 1) / kBlock;
  if (b > 8192) b = 8192;
  return b < 1 ? 1 : (int)b;
}

}  // namespace

void launch_visco(int dim, int all, const ViscoConst& c, const ViscoFields& f, hipStream_t s) {
  const int b = blocks_for(f.n);
#define TV_V(D, A) hipLaunchKernelGGL((k_visco_fused<D, A>), dim3(b), dim3(kBlock), 0, s, c, f)
  if (dim == 1) { if (all) TV_V(1, true); else TV_V(1, false); }
  else if (dim == 2) { if (all) TV_V(2, true); else TV_V(2, false); }
  else { if (all) TV_V(3, true); else TV_V(3, false); }
#undef TV_V
}

void launch_copy_gated(double* dst, const double* src, int64_t n, const NewtonGate& g, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_copy_gated, dim3(blocks_for(n)), dim3(kBlock), 0, s, dst, src, n, g);
}

void launch_visco_Tpass(int dim, int all, const ViscoConst& c, const ViscoFields& f, hipStream_t s) {
  (void)dim;
  const int b = blocks_for(f.n);
  if (all) hipLaunchKernelGGL((k_visco_T<true>), dim3(b), dim3(kBlock), 0, s, c, f);
  else hipLaunchKernelGGL((k_visco_T<false>), dim3(b), dim3(kBlock), 0, s, c, f);
}

void launch_visco_Spass(int dim, int all, const ViscoConst& c, const ViscoFields& f, hipStream_t s) {
  const int b = blocks_for(f.n);
#define TV_V(D, A) hipLaunchKernelGGL((k_visco_S<D, A>), dim3(b), dim3(kBlock), 0, s, c, f)
  if (dim == 1) { if (all) TV_V(1, true); else TV_V(1, false); }
  else if (dim == 2) { if (all) TV_V(2, true); else TV_V(2, false); }
  else { if (all) TV_V(3, true); else TV_V(3, false); }
#undef TV_V
}

}  // namespace tv
