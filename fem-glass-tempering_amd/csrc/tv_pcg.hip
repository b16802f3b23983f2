// Jacobi-preconditioned CG vector kernels, deterministic reductions and the
// device-side scalar logic of PETSc KSPCG (preconditioned norm, zero initial
// guess) + KSPConvergedDefault, gfx950.
//
// Replaces PETSc VecAXPY / VecAYPX / VecNorm / VecXDot / PCApply(Jacobi) and the
// KSPSolve_CG control flow that the reference runs inside dolfinx's Newton
// solver (ThermoViscoProblem.py:339-346).  All scalars live on the device
// (PcgState) so a batch of iterations is launched without host round trips;
// once converged every kernel of the batch exits at its first instruction.
// Reductions: per-block partial sums (fixed order) -> one-block reduce, so the
// result is bitwise reproducible run to run.
#include <algorithm>
#include <cstdlib>

#include "tv_device.h"

namespace tv {
namespace {

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

template <int W>
__device__ __forceinline__ void block_partials(double (&v)[W], double* partials) {
  __shared__ double red[W][kBlock / kWave];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int w = 0; w < W; ++w) {
    const double s = wave_sum(v[w]);
    if (lane == 0) red[w][wave] = s;
  }
  __syncthreads();
  if (threadIdx.x < W) {
    const int w = threadIdx.x;
    store_partial(&partials[(int64_t)blockIdx.x * W + w], (red[w][0] + red[w][1]) + (red[w][2] + red[w][3]));
  }
}

__global__ __launch_bounds__(kBlock) void k_pcg_init(int64_t n, const double* __restrict__ r,
                                                     const double* __restrict__ dinv, double* __restrict__ z,
                                                     double* __restrict__ dx, double* __restrict__ partials) {
  double acc[2] = {0.0, 0.0};
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < n; t += (int64_t)gridDim.x * kBlock) {
    const double rr = r[t];
    const double zz = dinv[t] * rr;  // PCApply (Jacobi)
    z[t] = zz;
    dx[t] = 0.0;
    acc[0] += zz * zz;
    acc[1] += zz * rr;
  }
  block_partials<2>(acc, partials);
}

// Cache policy of the update's streams (template bits, 7 in production): 1 = w, dx,
// p_prev loads non-temporal, 2 = dx stores non-temporal, 4 = dinv load
// non-temporal.  Only p (the next matvec's p_old) and z (its input) are written
// or read with the default policy, so they are what the Infinity Cache keeps
// between the two launches of a PCG iteration: measured inside the iteration
// (tv_time_kernel 5 / 6) the fused matvec drops from 92 to 70 us and the update
// from 103 to 90 us (C4, MI355X).
template <bool NTL>
__device__ __forceinline__ double ldc(const double* p) { return NTL ? __builtin_nontemporal_load(p) : *p; }
template <bool NTS>
__device__ __forceinline__ void stc(double* p, double v) {
  if (NTS) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// DXU: odd iteration, applies the dx steps of this and the previous iteration.
// Streams: w, dinv (+ p_prev, p, dx) read, z read and written (+ dx written):
// 32 B per node on even iterations, 64 B on odd ones.
// rt.lag (multi-rank): the alpha logic on the all-reduced p.w runs lagged
// here (lagged_state) and the tail commits it.
template <bool FACES, int NT, bool DXU>
__global__ __launch_bounds__(kBlock) void k_pcg_update(int64_t n, const PcgState* __restrict__ st,
                                                       const double* __restrict__ pA,
                                                       const double* __restrict__ pB,
                                                       const double* __restrict__ w,
                                                       const double* __restrict__ dinv, double* __restrict__ dx,
                                                       double* __restrict__ z, double* __restrict__ partials,
                                                       RedTail rt, FaceAdd fa, int it_host) {
  stamp_start(rt);
  double a, ap;
  if (rt.lag != nullptr) {
    const PcgState ls = lagged_state(st, rt.lag, rt.lag_kind);
    if (ls.done) { commit_done(rt.st, ls); return; }  // (rt.st == st; st stays read-only)
    a = ls.a;
    ap = DXU ? ls.a_prev : 0.0;
  } else {
    if (st->done) return;
    a = st->a;
    ap = DXU ? st->a_prev : 0.0;
  }
  const double* __restrict__ p = (it_host & 1) ? pB : pA;   // this iteration's p (== st->it parity)
  const double* __restrict__ pp = (it_host & 1) ? pA : pB;  // the previous iteration's
  constexpr bool NT1 = (NT & 1) != 0, NT2 = (NT & 2) != 0, NT4 = (NT & 4) != 0;
  double acc[2] = {0.0, 0.0};
  // one node: v = {w, dinv, z, dx, p_prev, p} as loaded
  auto node = [&](int64_t q, const double (&v)[6]) {
    if (DXU) stc<NT2>(&dx[q], (v[3] + ap * v[4]) + a * v[5]);  // x <- (x + a_prev p_prev) + a p
    double wt = v[0];
    if (FACES) wt += face_terms(fa, q);  // w = J p incl. the Robin facet terms
    // r <- r - a w, r = B^-1 z; B = 0 on Dirichlet-constrained nodes (z stays 0)
    const double rr = (v[1] != 0.0 ? v[2] / v[1] : 0.0) - a * wt;
    const double zz = v[1] * rr;             // z <- B r
    z[q] = zz;
    acc[0] += zz * zz;
    acc[1] += zz * rr;
  };
  auto load = [&](int64_t q, double (&v)[6]) {
    v[0] = ldc<NT1>(&w[q]);
    v[1] = ldc<NT4>(&dinv[q]);
    v[2] = z[q];
    if (DXU) {
      v[3] = ldc<NT1>(&dx[q]);
      v[4] = ldc<NT1>(&pp[q]);
      v[5] = p[q];
    }
  };
  // U nodes per thread and round, every load of the round issued before the
  // first store: 3 (6) loads per node alone leave too few bytes in flight
  constexpr int U = 4;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x;
  for (; t + (U - 1) * stride < n; t += U * stride) {
    double v[U][6];
#pragma unroll
    for (int u = 0; u < U; ++u) load(t + u * stride, v[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) node(t + u * stride, v[u]);
  }
  for (; t < n; t += stride) {
    double v[6];
    load(t, v);
    node(t, v);
  }
  block_partials<2>(acc, partials);
  fused_reduce_tail<2>(rt, gridDim.x);
}

// ---- multigrid-preconditioned CG: level-0 vector kernels --------------------
// KSPCG update with an explicit residual (the V-cycle smooths against r):
// r <- r - a (w + facet terms), dx <- dx + a p, and the V-cycle's first
// pre-smoothing step from 0, x0 <- omega dinv r.  INIT: dx <- 0, x0 <- omega dinv r.
// DXU (odd iterations): dx <- (dx + a_prev p_prev) + a p, the steps of this
// and the previous iteration (both p buffers are live until the next matvec),
// so the dx stream moves every second iteration only: 40 B per node on even
// iterations, 72 on odd ones (56 mean, was 64); a solve of odd length ends
// with k_dx_tail.  U nodes per thread and round, every load issued first.
// FIRST (iteration 1, the first DXU one): dx is assigned, not accumulated, so
// the init pass does not have to zero it (mg_dx_finish covers solves of 0 / 1
// iterations)
// lag != nullptr (multi-rank): the alpha logic (kind 2) on the all-reduced
// p.w is formed here (lagged_state) and committed by the last workgroup to
// arrive at `counter` -- no one-thread logic launch between the all-reduce
// and this update.
template <bool FACES, bool INIT, bool DXU, bool FIRST = false>
__global__ __launch_bounds__(kBlock) void k_mg_update(int64_t n, const PcgState* __restrict__ st,
                                                      const double* __restrict__ pA, const double* __restrict__ pB,
                                                      const double* __restrict__ w, FaceAdd fa,
                                                      const double* __restrict__ dinv, double omega,
                                                      double* __restrict__ r, double* __restrict__ dx,
                                                      double* __restrict__ x0, int it_host, const double* lag,
                                                      unsigned* counter, PcgState* st_w) {
  double a = 0.0, ap = 0.0;
  if (!INIT && lag != nullptr) {
    const PcgState ls = lagged_state(st, lag, 2);
    if (ls.done) { commit_done(st_w, ls); return; }  // st_w == st (writes only through it)
    a = ls.a;
    ap = DXU ? ls.a_prev : 0.0;
  } else {
    if (st->done) return;
    a = INIT ? 0.0 : st->a;
    ap = DXU ? st->a_prev : 0.0;
  }
  const double* __restrict__ p = (it_host & 1) ? pB : pA;
  const double* __restrict__ pp = (it_host & 1) ? pA : pB;
  // v = {r, w, dinv, dx, p_prev, p}.  (D^-1 formed on the fly from the axis
  // tables instead of this stream -- 8 B per node fewer -- measured slower:
  // C4 10.72 / 10.77 vs 10.71 / 10.66 ms, the per-lane index decode, table
  // gathers and the divide cost more than the stream)
  auto load = [&](int64_t q, double (&v)[6]) {
    v[0] = r[q];
    v[2] = ldc<true>(&dinv[q]);
    if (!INIT) v[1] = ldc<true>(&w[q]);
    if (DXU) {
      v[3] = FIRST ? 0.0 : ldc<true>(&dx[q]);
      v[4] = ldc<true>(&pp[q]);
      v[5] = ldc<true>(&p[q]);
    }
  };
  auto node = [&](int64_t q, const double (&v)[6]) {
    double rr = v[0];
    if (INIT) {
      // dx is left alone: iteration 1 assigns it (FIRST)
    } else {
      double wt = v[1];
      if (FACES) wt += face_terms(fa, q);
      rr -= a * wt;
      r[q] = rr;
      if (DXU) stc<true>(&dx[q], (v[3] + ap * v[4]) + a * v[5]);
    }
    x0[q] = omega * v[2] * rr;
  };
  constexpr int U = 4;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x;
  for (; t + (U - 1) * stride < n; t += U * stride) {
    double v[U][6];
#pragma unroll
    for (int u = 0; u < U; ++u) load(t + u * stride, v[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) node(t + u * stride, v[u]);
  }
  for (; t < n; t += stride) {
    double v[6];
    load(t, v);
    node(t, v);
  }
  if (!INIT && lag != nullptr && last_block_arrived(counter, gridDim.x) && threadIdx.x == 0) {
    const PcgState ls = lagged_state(st, lag, 2);  // formed again (see lagged_state)
    *st_w = ls;
  }
}

// The single-reduction (Chronopoulos-Gear) form of the multigrid-preconditioned
// CG on a deep-ghost slab (tv_mgdist.cpp): after the V-cycle (z = M r, z.z and
// z.r) and the matvec (u = A z complete, z.u) ONE all-reduce of the three sums
// closes an iteration, and this launch forms the scalars from them (lagged
// kind 6, or 7 at iteration 0) and applies
//   s <- u + beta s,  p <- z + beta p,  dx <- dx + a p,  r <- r - a s,
//   x0 <- omega dinv r  (the next V-cycle's pre-smoothing from 0)
// FIRST (iteration 0): s = u, p = z, dx = a p.  96 B per node.  Runs over the
// write window (r, s and x0 are needed on the ghost planes; p and dx are only
// read on the owned ones).
template <bool FIRST>
__global__ __launch_bounds__(kBlock) void k_mg_update_cgs(int64_t n, const PcgState* __restrict__ st,
                                                          const double* __restrict__ u, double* __restrict__ s,
                                                          const double* __restrict__ z, double* __restrict__ p,
                                                          double* __restrict__ dx, double* __restrict__ r,
                                                          const double* __restrict__ dinv, double omega,
                                                          double* __restrict__ x0, const double* lag, int lag_kind,
                                                          unsigned* counter, PcgState* st_w) {
  double a, beta;
  if (lag != nullptr) {
    const PcgState ls = lagged_state(st, lag, lag_kind);
    if (ls.done) { commit_done(st_w, ls); return; }
    a = ls.a;
    beta = ls.beta;
  } else {
    if (st->done) return;
    a = st->a;
    beta = st->beta;
  }
  constexpr int U = 2;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x;
  auto node = [&](int64_t q, const double (&v)[7]) {  // v = {u, s, z, p, dx, r, dinv}
    const double sn = FIRST ? v[0] : v[0] + beta * v[1];
    const double pn = FIRST ? v[2] : v[2] + beta * v[3];
    const double rn = v[5] - a * sn;
    s[q] = sn;
    p[q] = pn;
    __builtin_nontemporal_store(FIRST ? a * pn : v[4] + a * pn, &dx[q]);
    r[q] = rn;
    x0[q] = omega * v[6] * rn;
  };
  auto load = [&](int64_t q, double (&v)[7]) {
    v[0] = __builtin_nontemporal_load(&u[q]);
    v[1] = FIRST ? 0.0 : s[q];
    v[2] = __builtin_nontemporal_load(&z[q]);
    v[3] = FIRST ? 0.0 : p[q];
    v[4] = FIRST ? 0.0 : __builtin_nontemporal_load(&dx[q]);
    v[5] = r[q];
    v[6] = __builtin_nontemporal_load(&dinv[q]);
  };
  for (; t + (U - 1) * stride < n; t += U * stride) {
    double v[U][7];
#pragma unroll
    for (int k = 0; k < U; ++k) load(t + k * stride, v[k]);
#pragma unroll
    for (int k = 0; k < U; ++k) node(t + k * stride, v[k]);
  }
  for (; t < n; t += stride) {
    double v[7];
    load(t, v);
    node(t, v);
  }
  if (lag != nullptr && last_block_arrived(counter, gridDim.x) && threadIdx.x == 0) *st_w = lagged_state(st, lag, lag_kind);
}

// post-smoothing of level 0: z <- x0 + omega dinv (r - w), w = J x0; (z.z,
// z.r) records and the KSPCG logic in the reduction tail (init: kind 1)
template <bool FACES>
__global__ __launch_bounds__(kBlock) void k_mg_post(int64_t n, const PcgState* __restrict__ st,
                                                    const double* __restrict__ x0, const double* __restrict__ r,
                                                    const double* __restrict__ w, FaceAdd fa,
                                                    const double* __restrict__ dinv, double omega,
                                                    double* __restrict__ z, double* __restrict__ partials,
                                                    RedTail rt) {
  if (st->done) return;
  double acc[2] = {0.0, 0.0};
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < n; t += (int64_t)gridDim.x * kBlock) {
    const double rr = r[t];
    double wt = w[t];
    if (FACES) wt += face_terms(fa, t);
    const double zz = x0[t] + omega * dinv[t] * (rr - wt);
    z[t] = zz;
    acc[0] += zz * zz;
    acc[1] += zz * rr;
  }
  block_partials<2>(acc, partials);
  fused_reduce_tail<2>(rt, gridDim.x);
}

__global__ __launch_bounds__(kBlock) void k_dx_tail(int64_t n, const PcgState* __restrict__ st,
                                                    const double* __restrict__ p, double* __restrict__ dx) {
  const double a = st->a;
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < n; t += (int64_t)gridDim.x * kBlock)
    dx[t] += a * p[t];
}

// the post-solve group of a Newton iteration queued behind every batch of a
// multigrid solve (pcg_solve_mg): it runs once, behind the batch that ends
// the solve, so the host's convergence poll overlaps it -- and only when the
// solve ended well (converged, or the fixed iteration count of ksp_fixed_its):
// a diverged solve (NaN / Inf, DTOL, indefinite, DIVERGED_ITS) leaves T and dx
// untouched, and newton() then returns TV_ERR_KSP with the state as it was
__device__ __forceinline__ bool post_gate(const PcgState* st) {
  const bool good = st->reason > 0 || (st->reason == R_DIV_ITS && st->accept_its);
  return st->done && !st->post && good;
}

__global__ __launch_bounds__(kBlock) void k_newton_update(int64_t n, double* __restrict__ T,
                                                          const double* __restrict__ dx,
                                                          double* __restrict__ partials, RedTail rt,
                                                          const PcgState* __restrict__ gate) {
  if (gate != nullptr && !post_gate(gate)) return;
  double acc[1] = {0.0};
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < n; t += (int64_t)gridDim.x * kBlock) {
    const double d = dx[t];
    T[t] -= d;  // x <- x - relaxation * dx   (relaxation 1)
    acc[0] += d * d;
  }
  block_partials<1>(acc, partials);
  fused_reduce_tail<1>(rt, gridDim.x);  // ||dx||^2 into rt.out (one partition: no separate reduce launch)
}

// the post-solve group in one pass: dx after the solve, from the device's
// iteration count (pA == nullptr: the single-reduction form, whose updates keep
// dx complete -- only a solve that converged at its start leaves dx to zero),
// and k_newton_update's T <- T - dx with the ||dx||^2 records, the same values
// and the same records (one launch and one dx read fewer per Newton iteration)
__global__ __launch_bounds__(kBlock) void k_post_fused(int64_t n, const PcgState* __restrict__ st,
                                                       const double* __restrict__ pA, const double* __restrict__ pB,
                                                       double* __restrict__ dx, double* __restrict__ T,
                                                       double* __restrict__ partials) {
  if (!post_gate(st)) return;
  const int its = st->it;
  const double a = st->a;
  // 0: dx as stored; 1: dx <- 0; 2: dx <- a pA; 3: dx <- dx + a p (the odd tail)
  int mode = 0;
  const double* __restrict__ p = pA;
  if (pA == nullptr) {
    if (its == 0) mode = 1;
  } else if (its <= 1) {
    mode = its == 0 ? 1 : 2;
  } else if (its & 1) {
    mode = 3;
    p = ((its - 1) & 1) ? pB : pA;
  }
  double acc[1] = {0.0};
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < n; t += (int64_t)gridDim.x * kBlock) {
    double d;
    if (mode == 0) {
      d = dx[t];
    } else {
      d = mode == 1 ? 0.0 : (mode == 2 ? a * p[t] : dx[t] + a * p[t]);
      dx[t] = d;
    }
    T[t] -= d;  // x <- x - relaxation * dx   (relaxation 1)
    acc[0] += d * d;
  }
  block_partials<1>(acc, partials);
}

// One-block deterministic reduction of `n` partial records of width W, then
// (optionally) the scalar logic.  kind: 0 none, 1 init, 2 dpi, 3 update.
__global__ __launch_bounds__(1024) void k_reduce(const double* __restrict__ partials, int n, int W,
                                                 double* __restrict__ out, PcgState* st, int kind,
                                                 int check_done) {
  // check_done 2: the post-solve group's norm (post_gate), which marks the group as run
  if (check_done == 2 ? !post_gate(st) : (check_done && st->done)) return;
  __shared__ double red[2][16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double acc[2] = {0.0, 0.0};
  for (int t = threadIdx.x; t < n; t += blockDim.x) {
    acc[0] += partials[(int64_t)t * W];
    if (W > 1) acc[1] += partials[(int64_t)t * W + 1];
  }
  for (int w = 0; w < W; ++w) {
    const double s = wave_sum(acc[w]);
    if (lane == 0) red[w][wave] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double sums[2] = {0.0, 0.0};
    const int nw = blockDim.x >> 6;
    for (int w = 0; w < W; ++w) {
      double s = 0.0;
      for (int q = 0; q < nw; ++q) s += red[w][q];
      sums[w] = s;
      out[w] = s;
    }
    apply_logic(st, sums, kind);
    if (check_done == 2) st->post = 1;
  }
}

__global__ void k_logic(PcgState* st, const double* sums, int kind) { apply_logic(st, sums, kind); }
__global__ void k_set_state(PcgState* st, PcgState h, const double* __restrict__ gate) {
  if (gate != nullptr && *gate != 0.0) {
    h.done = 1;
    h.reason = R_SKIPPED;
  }
  *st = h;
}

__global__ __launch_bounds__(kBlock) void k_fill(double* x, int64_t n, double v) {
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < n; t += (int64_t)gridDim.x * kBlock) x[t] = v;
}
__global__ __launch_bounds__(kBlock) void k_copy(double* __restrict__ d, const double* __restrict__ s, int64_t n) {
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < n; t += (int64_t)gridDim.x * kBlock) d[t] = s[t];
}

int vec_blocks(int64_t n) {
  int64_t b = (n + kBlock - 1) / kBlock;
  // default: at least kVecNodesPerThread nodes per thread (four 4-node rounds of
  // the PCG update), between kVecBlocksMin and kVecBlocks workgroups.  Fewer
  // workgroups than one node per thread cut the partial records the reduction
  // tail walks: 19-20 -> 15.5 us per update at 1M nodes (the per-GPU share of C4
  // on 8 GPUs; 256 workgroups measured at or below 512 on every box, 128 worse);
  // at C4 on one GPU the cap of 1024 still holds.  (8 nodes per thread and load
  // round instead of 4: no gain at 1M nodes or at C4.)
  const int64_t lim = std::min<int64_t>(kVecBlocks, std::max<int64_t>(kVecBlocksMin,
      (n + (int64_t)kBlock * kVecNodesPerThread - 1) / ((int64_t)kBlock * kVecNodesPerThread)));
  if (b > lim) b = lim;
  return b < 1 ? 1 : (int)b;
}

}  // namespace

int pcg_vec_blocks(int64_t n) { return vec_blocks(n); }

void launch_pcg_init(int64_t n, const double* r, const double* dinv, double* z, double* dx, double* partials,
                     hipStream_t s) {
  hipLaunchKernelGGL(k_pcg_init, dim3(vec_blocks(n)), dim3(kBlock), 0, s, n, r, dinv, z, dx, partials);
}

void launch_mg_update(int64_t n, const PcgState* st, const double* pA, const double* pB, const double* w,
                      const FaceAdd* fa, const double* dinv, double omega, double* r, double* dx, double* x0,
                      int it_host, int init, hipStream_t s, const double* lag, unsigned* counter) {
  const FaceAdd f = (fa && fa->on) ? *fa : FaceAdd{};
  const dim3 g(vec_blocks(n)), b(kBlock);
  const bool odd = (it_host & 1) != 0;
  const bool first = it_host == 1;
#define TV_MGU(F, I, D, FI) \
  hipLaunchKernelGGL((k_mg_update<F, I, D, FI>), g, b, 0, s, n, st, pA, pB, w, f, dinv, omega, r, dx, x0, it_host, \
                     lag, counter, const_cast<PcgState*>(st))
  if (init) TV_MGU(false, true, false, false);
  else if (f.on) {
    if (first) TV_MGU(true, false, true, true);
    else if (odd) TV_MGU(true, false, true, false);
    else TV_MGU(true, false, false, false);
  } else {
    if (first) TV_MGU(false, false, true, true);
    else if (odd) TV_MGU(false, false, true, false);
    else TV_MGU(false, false, false, false);
  }
#undef TV_MGU
}

int launch_mg_post(int64_t n, const PcgState* st, const double* x0, const double* r, const double* w,
                   const FaceAdd* fa, const double* dinv, double omega, double* z, double* partials,
                   const RedTail* tail, hipStream_t s) {
  const RedTail rt = tail ? *tail : RedTail{};
  const FaceAdd f = (fa && fa->on) ? *fa : FaceAdd{};
  const int nb = vec_blocks(n);
  if (f.on)
    hipLaunchKernelGGL(k_mg_post<true>, dim3(nb), dim3(kBlock), 0, s, n, st, x0, r, w, f, dinv, omega, z, partials, rt);
  else
    hipLaunchKernelGGL(k_mg_post<false>, dim3(nb), dim3(kBlock), 0, s, n, st, x0, r, w, f, dinv, omega, z, partials, rt);
  return nb;
}

void launch_mg_update_cgs(int64_t n, const PcgState* st, const double* u, double* s, const double* z, double* p,
                          double* dx, double* r, const double* dinv, double omega, double* x0, bool first,
                          const double* lag, int lag_kind, unsigned* counter, hipStream_t stream) {
  const dim3 g(vec_blocks(n)), b(kBlock);
  PcgState* stw = const_cast<PcgState*>(st);
  if (first)
    hipLaunchKernelGGL(k_mg_update_cgs<true>, g, b, 0, stream, n, st, u, s, z, p, dx, r, dinv, omega, x0, lag, lag_kind,
                       counter, stw);
  else
    hipLaunchKernelGGL(k_mg_update_cgs<false>, g, b, 0, stream, n, st, u, s, z, p, dx, r, dinv, omega, x0, lag, lag_kind,
                       counter, stw);
}

void launch_pcg_update(int64_t n, PcgState* st, const double* pA, const double* pB, const double* w,
                       const double* dinv, double* dx, double* z, double* partials, hipStream_t s,
                       const RedTail* tail, const FaceAdd* fa, int it_host) {
  RedTail rt{};
  if (tail) rt = *tail;
  // non-temporal policy (7) on w, dinv, dx, p_prev: the Infinity Cache keeps z
  // and p for the next matvec (measured against the default policy, round 1)
  const FaceAdd f = (fa && fa->on) ? *fa : FaceAdd{};
  const int v = (fa && fa->on ? 2 : 0) | (it_host & 1);
#define TV_UPD(F, D)                                                                                          \
  hipLaunchKernelGGL((k_pcg_update<F, 7, D>), dim3(vec_blocks(n)), dim3(kBlock), 0, s, n, st, pA, pB, w, dinv, \
                     dx, z, partials, rt, f, it_host);                                                          \
  break
  switch (v) {
    case 0: TV_UPD(false, false);
    case 1: TV_UPD(false, true);
    case 2: TV_UPD(true, false);
    default: TV_UPD(true, true);
  }
#undef TV_UPD
}

__global__ __launch_bounds__(kBlock) void k_dx_set(int64_t n, const PcgState* __restrict__ st,
                                                  const double* __restrict__ p, double* __restrict__ dx) {
  const double a = p != nullptr ? st->a : 0.0;
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < n; t += (int64_t)gridDim.x * kBlock)
    dx[t] = p != nullptr ? a * p[t] : 0.0;
}

void launch_mg_dx_finish(int64_t n, const PcgState* st, const double* pA, const double* pB, double* dx, int its,
                         hipStream_t s) {
  if (its == 0)  // converged at the init: dx = 0
    hipLaunchKernelGGL(k_dx_set, dim3(vec_blocks(n)), dim3(kBlock), 0, s, n, st, nullptr, dx);
  else if (its == 1)  // iteration 0 only: dx was never assigned
    hipLaunchKernelGGL(k_dx_set, dim3(vec_blocks(n)), dim3(kBlock), 0, s, n, st, pA, dx);
  else
    launch_pcg_dx_tail(n, st, pA, pB, dx, its, s);
}

void launch_pcg_dx_tail(int64_t n, const PcgState* st, const double* pA, const double* pB, double* dx, int its,
                        hipStream_t s) {
  if (!(its & 1)) return;
  hipLaunchKernelGGL(k_dx_tail, dim3(vec_blocks(n)), dim3(kBlock), 0, s, n, st, (its - 1) & 1 ? pB : pA, dx);
}

void launch_newton_update(int64_t n, double* T, const double* dx, double* partials, hipStream_t s,
                          const RedTail* tail) {
  const RedTail rt = tail ? *tail : RedTail{};
  hipLaunchKernelGGL(k_newton_update, dim3(vec_blocks(n)), dim3(kBlock), 0, s, n, T, dx, partials, rt,
                     static_cast<const PcgState*>(nullptr));
}

void launch_post_group(int64_t n, const PcgState* st, const double* pA, const double* pB, double* dx, double* T,
                       double* partials, double* sums, hipStream_t s) {
  hipLaunchKernelGGL(k_post_fused, dim3(vec_blocks(n)), dim3(kBlock), 0, s, n, st, pA, pB, dx, T, partials);
  hipLaunchKernelGGL(k_reduce, dim3(1), dim3(1024), 0, s, partials, vec_blocks(n), 1, sums, const_cast<PcgState*>(st), 0,
                     2);
}

void launch_reduce_logic(const double* partials, int n, int W, double* out, PcgState* st, int kind,
                         int check_done, hipStream_t s) {
  hipLaunchKernelGGL(k_reduce, dim3(1), dim3(1024), 0, s, partials, n, W, out, st, kind, check_done);
}

// the solver state at a solve's start, by a one-thread launch rather than a
// host-to-device copy: the copy of a pinned 160-byte struct was followed by a
// ~45 us gap before the next kernel in the C4 trace (the runtime's copy path),
// a launch is queued like every other kernel
void launch_set_state(PcgState* st, const PcgState& h, hipStream_t s, const double* gate) {
  hipLaunchKernelGGL(k_set_state, dim3(1), dim3(1), 0, s, st, h, gate);
}

void launch_logic(PcgState* st, const double* sums, int kind, hipStream_t s) {
  hipLaunchKernelGGL(k_logic, dim3(1), dim3(1), 0, s, st, sums, kind);
}

void launch_fill(double* x, int64_t n, double v, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_fill, dim3(vec_blocks(n)), dim3(kBlock), 0, s, x, n, v);
}

void launch_copy(double* dst, const double* src, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_copy, dim3(vec_blocks(n)), dim3(kBlock), 0, s, dst, src, n);
}

}  // namespace tv
