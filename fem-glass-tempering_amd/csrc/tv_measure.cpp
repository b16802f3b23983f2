// Measurement entry points: in-solve kernel timing from device clock stamps,
// algorithmic bytes per launch and timed launches of the
// hot kernels (HIP events), including the Infinity-Cache-flushed J x.
#include <algorithm>

#include "tv_ctx.h"

namespace tv {
// read-only sweep (cache state for the flushed timing of tv_time_kernel id 10):
// one sum per workgroup into out[block] so the loads are not dead
__global__ __launch_bounds__(kBlock) void k_read_sweep(const double* __restrict__ a, int64_t n, double* out) {
  double acc = 0.0;
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < n; t += (int64_t)gridDim.x * kBlock) acc += a[t];
  if (acc == 12345.678) out[blockIdx.x] = acc;  // practically never: keeps the loads
}
// launch audit (tv_time_kernel ids 12-17): a one-thread kernel that holds the
// stream for `ticks` of the 100 MHz REALTIME clock, so that the chain queued
// behind it is timed as the GPU runs it, not at the host's enqueue rate
__global__ void k_spin(uint64_t ticks) {
  if (threadIdx.x == 0) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(16);
  }
}
__global__ void k_noop() {}

}  // namespace tv

using namespace tv;

extern "C" {

int tv_kernel_bytes(void* ctx, int kernel, double* bytes) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c || !bytes) return TV_ERR_ARG;
  const double n = (double)c->ownT_n;
  const int dd = c->dim * c->dim;
  switch (kernel) {
    case 0:  // J(T) x : read x, write y (geometry implicit, T only on boundary nodes)
    case 10:  // the same, timed with the Infinity Cache flushed (tv_time_kernel)
      // unstructured: + the assembled operator -- structured topology: the 14
      // upper stencil slots of J(T) per row (112 B; the lower slots are the
      // neighbour rows' upper slots, counted once); else 8 B value + 4 B column
      // per stored SELL entry, padding included
      *bytes = !c->um ? 16.0 * n
                      : (c->umg.J14 ? (16.0 + 112.0) * n : 16.0 * n + 12.0 * (double)um_nnz(c->umd));
      break;
    case 1: {  // fused visco update, per dof
      int tf = 1;
      HIPC(hipMemcpy(&tf, c->tflag, sizeof(int), hipMemcpyDeviceToHost));
      const int tilde = tf ? 2 * 6 * dd : 0;  // s~, sigma~ are not touched while they are all +0.0
      double per = 8.0 * (2 + 6 + tilde)            // read T, Tp, Tf_partial (, s~, sigma~)
                   + 8.0 * (6 + 3 + tilde + dd);    // write Tf_partial, Tf, phi, xi (, s~, sigma~), sigma
      if (c->O.materialize) per += 8.0 * (2 + 3 * dd + 4 * 6 * dd);
      *bytes = per * n;
      break;
    }
    case 2:  // residual: read T, Tp, write F
      *bytes = 24.0 * n;
      break;
    case 3:  // fused PCG matvec: read z, p_old, write p, w (T on boundary nodes only)
      // single-reduction iteration: read r, s, w, diag^-1, p, x; write r, s, p, x, w
      *bytes = (c->cgs ? 88.0 : 32.0) * n;
      break;
    case 5:
    case 7:
      *bytes = 32.0 * n;
      break;
    case 4:  // PCG update, mean of an even / odd pair: read w, dinv, z, write z (+ odd: read p_prev, p, dx, write dx)
      *bytes = c->cgs ? 0.0 : 48.0 * n;
      break;
    case 6:
    case 8:
      *bytes = 48.0 * n;
      break;
    case 11: {  // one multigrid V-cycle, per node of each level (streams counted once)
      if (!c->mg_on) return c->fail(TV_ERR_ARG, "kernel 11: preconditioner GMG not enabled");
      if (c->amg_on) {  // the algebraic cycle: stored operator entries + vector streams
        *bytes = amg_cycle_bytes(c);
        break;
      }
      // level 0: J x0 (16), restriction reads r, w (16), prolongation x0 -> x (16),
      // then CG: J x with the post-smoothing in its epilogue (x, r in, z out: 24;
      // D^-1 formed in the kernel off the physical boundary),
      // DG: J x (16) + the cell-block post-smoothing (x0, r, w in, z out: 32)
      // (a fused residual restriction, RRArgs: no J x0, the restriction reads r
      // and x0 -- 16 B instead of 32; the facet terms it needs touch the faces only)
      const bool rr0 = !c->mg_dg && !c->mg.empty() && c->mg[0].rr.on;
      double b = (c->mg_dg ? 16.0 + 16 + 16 + 16 + 32 : (rr0 ? 0.0 : 16.0) + 16 + 16 + 24) * n;
      for (size_t l = 0; l < c->mg.size(); ++l) {
        const double nl = (double)c->mg[l].n;
        b += 24.0 * nl;  // the restriction's outputs b, x (pre-smoothing) and the dinv it reads
        const bool rr = l + 1 < c->mg.size() && c->mg[l + 1].rr.on;
        if (l + 1 < c->mg.size())  // J x (16), restriction reads (16), partial J x (16), prolongation in (16),
          b += ((rr ? 0.0 : 16.0) + 16 + 16 + 16 + 24) * nl;  // post-smoothing operands b, w, dinv (24)
      }
      *bytes = b;
      break;
    }
    default:
      return c->fail(TV_ERR_ARG, "unknown kernel id");
  }
  return TV_OK;
}


int tv_time_kernel(void* ctx, int kernel, int reps, double* ms) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c || !ms || reps < 1) return TV_ERR_ARG;
  hipSetDevice(c->device);
  if (kernel == 4 && c->cgs) return c->fail(TV_ERR_ARG, "kernel 4: no separate update in the single-reduction PCG");
  if (kernel >= 3 && kernel <= 8) {  // PCG kernels need a running solver state
    PcgState h{};
    h.beta = 1.0; h.betaold = 2.0; h.a = 1e-3; h.it = 1; h.done = 0; h.max_it = 1 << 30;
    h.gamma = 1.0; h.eta = 1.0;
    HIPC(hipMemcpyAsync(c->st, &h, sizeof(PcgState), hipMemcpyHostToDevice, c->stream));
  }
  int upd_it = 0;
  // the J x of a solve: on a structured-topology unstructured mesh the Robin
  // terms at the current T are folded into the stencil once (as each Newton
  // iteration does), and the matvec alone is timed
  if (c->um && (kernel == 0 || kernel == 10)) launch_um_robin_fold(c->umg, c->f[TV_F_T].ptr, c->stream);
  auto jx = [&]() {
    if (c->um) launch_um_japply(c->umg, c->f[TV_F_T].ptr, c->pA, c->w, c->stream);
    else op_japply(c, c->f[TV_F_T].ptr, c->pA, c->w, nullptr, nullptr);
  };
  if (kernel == 11) {  // V-cycles on the current state (solver state reset: not converged)
    if (!c->mg_on) return c->fail(TV_ERR_ARG, "kernel 11: preconditioner GMG not enabled");
    PcgState h{};
    h.max_it = 1 << 30;
    HIPC(hipMemcpyAsync(c->st, &h, sizeof(PcgState), hipMemcpyHostToDevice, c->stream));
    if (c->n_parts > 1) {
      if (int e = mg_prepare_dist(c, c->f[TV_F_T].ptr)) return e;
    } else {
      if (int e = mg_prepare(c, c->f[TV_F_T].ptr)) return e;
    }
    if (int e = mg_dg_weight(c, c->f[TV_F_T].ptr)) return e;
  }
  auto one = [&]() -> int {
    int np = 0;
    switch (kernel) {
      case 11:  // partitioned: the distributed V-cycle, its exchanges included (every rank calls this)
        if (c->n_parts > 1) return mg_apply0_dist(c, c->f[TV_F_T].ptr, nullptr);
        mg_apply0(c, c->f[TV_F_T].ptr, nullptr);
        return TV_OK;
      case 0: jx(); return TV_OK;
      case 1: return visco(c, false);
      case 2: op_residual(c, c->f[TV_F_T].ptr, c->f[TV_F_T_PREV].ptr, c->r); return TV_OK;
      case 3:
        if (c->cgs) {  // the single-reduction iteration, parities alternating, no tail
          const int it = 2 + (upd_it++);
          const CgsBuffers v = cgs_buffers(c, c->f[TV_F_T].ptr, it);
          launch_cg_cgs(c->cg, false, v, c->st, c->partials, c->stream, nullptr, it, nullptr);
          return TV_OK;
        }
        op_japply_fused(c, c->f[TV_F_T].ptr, &np, nullptr, 1);  // st->it = 1 below
        return TV_OK;
      case 4: {
        const FaceAdd fa = (c->fam_T == TV_CG && !c->um) ? cg_face_add(c->cg, c->ownT_off) : FaceAdd{};
        launch_pcg_update(c->ownT_n, c->st, c->pA + c->ownT_off, c->pB + c->ownT_off, c->w + c->ownT_off,
                          c->dinv + c->ownT_off, c->f[TV_F_DX].ptr + c->ownT_off, c->z + c->ownT_off,
                          c->partials, c->stream, nullptr, &fa, upd_it++);  // even / odd alternate
        return TV_OK;
      }
      default: return c->fail(TV_ERR_ARG, "unknown kernel id");
    }
  };
  if (kernel >= 5 && kernel <= 8) {
    // matvec / update timed inside whole PCG iterations (march then update,
    // alternating, as in the solve), with (5, 6) or without (7, 8) the
    // in-kernel reduction tails (kind 0: reduce only, the state is not touched)
    if (c->fam_T != TV_CG || c->um)
      return c->fail(TV_ERR_ARG, "kernel ids 5-8: CG temperature space on a rectilinear mesh only");
    const bool tails = kernel <= 6;
    std::vector<hipEvent_t> ev(3 * (size_t)(reps + 1));
    for (auto& e : ev) HIPC(hipEventCreate(&e));
    const FaceAdd fa = cg_face_add(c->cg, c->ownT_off);
    const int64_t off = c->ownT_off, n = c->ownT_n;
    int np = 0;
    for (int i = 0; i <= reps; ++i) {
      RedTail t1{tails ? c->counters : nullptr, c->partials, c->sums, c->st, 0};
      RedTail t2{tails ? c->counters + kTailCounters : nullptr, c->partials, c->sums, c->st, 0};
      HIPC(hipEventRecord(ev[3 * i], c->stream));
      op_japply_fused(c, c->f[TV_F_T].ptr, &np, &t1, i + 1);  // both parities, as in the solve
      HIPC(hipEventRecord(ev[3 * i + 1], c->stream));
      launch_pcg_update(n, c->st, c->pA + off, c->pB + off, c->w + off, c->dinv + off, c->f[TV_F_DX].ptr + off,
                        c->z + off, c->partials, c->stream, &t2, &fa, i + 1);
      HIPC(hipEventRecord(ev[3 * i + 2], c->stream));
    }
    HIPC(hipEventSynchronize(ev.back()));
    double sum = 0.0;
    const int k0 = (kernel == 5 || kernel == 7) ? 0 : 1;
    for (int i = 1; i <= reps; ++i) {  // rep 0 is the warm-up
      float t = 0.f;
      HIPC(hipEventElapsedTime(&t, ev[3 * i + k0], ev[3 * i + k0 + 1]));
      sum += t;
    }
    for (auto& e : ev) hipEventDestroy(e);
    *ms = sum / reps;
    return TV_OK;
  }
  if (kernel >= 12 && kernel <= 17) {
    // launch audit: `reps` back-to-back launches of one
    // kind queued behind k_spin, HIP events around the chain, per launch =
    // elapsed / reps -- the dependent-launch cost as the GPU pays it, unprofiled.
    //   12 an empty one-thread kernel        13 k_set_state (one thread, 160-B argument)
    //   14 the one-block reduce + KSPCG logic 15 k_mg_jacobi on the coarsest GMG level
    //   16 J x on GMG level 1 (march)        17 J x on the fine grid (march + faces)
    if ((kernel >= 15 && kernel <= 16) && (!c->mg_on || c->mg.empty() || c->amg_on || c->mg_dg))
      return c->fail(TV_ERR_ARG, "kernel ids 15-16: CG GMG levels required");
    if (kernel == 17 && (c->um || c->fam_T != TV_CG)) return c->fail(TV_ERR_ARG, "kernel 17: CG box mesh");
    PcgState h{};
    h.max_it = 1 << 30;  // running: the GMG kernels do their work
    HIPC(hipMemcpyAsync(c->st, &h, sizeof(PcgState), hipMemcpyHostToDevice, c->stream));
    auto launch = [&]() {
      switch (kernel) {
        case 12: hipLaunchKernelGGL(k_noop, dim3(1), dim3(64), 0, c->stream); break;
        case 13: launch_set_state(c->st, h, c->stream, nullptr); break;
        case 14: launch_reduce_logic(c->partials, 256, 2, c->sums, c->st, 0, 0, c->stream); break;
        case 15: {
          MgLevel& L = c->mg.back();
          launch_mg_jacobi(L.n, c->st, L.b, nullptr, nullptr, L.dinv, L.omega, L.x, 0, c->stream);
          break;
        }
        case 16: {
          MgLevel& L = c->mg[0];
          launch_cg_japply(L.g, L.T, L.x, L.w, nullptr, nullptr, c->stream, c->st);
          break;
        }
        default: op_japply(c, c->f[TV_F_T].ptr, c->pA, c->w, nullptr, nullptr); break;
      }
    };
    for (int i = 0; i < 3; ++i) launch();  // warm-up
    HIPC(hipStreamSynchronize(c->stream));
    // ~8 us of host enqueue per launch at most: the chain is queued before the spin ends
    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, c->stream, (uint64_t)reps * 800 + 20000);
    HIPC(hipEventRecord(c->ev0, c->stream));
    for (int i = 0; i < reps; ++i) launch();
    HIPC(hipEventRecord(c->ev1, c->stream));
    HIPC(hipEventSynchronize(c->ev1));
    float t = 0.f;
    HIPC(hipEventElapsedTime(&t, c->ev0, c->ev1));
    *ms = (double)t / reps;
    return TV_OK;
  }
  if (kernel == 10) {
    // J x with the Infinity Cache flushed before every launch: a 512 MiB write
    // (2x the 256 MiB L3) then a read sweep of the same buffer, so the cache
    // holds clean lines (no write-backs of the flush competing with the timed
    // launch), HIP events around each launch alone; the MEDIAN over the reps
    // (the HBM figure, not
    // the cache-assisted one).  The events include the dispatch (~6 us before
    // the first workgroup in a kernel trace).
    const size_t fl = (size_t)512 << 20;
    void* flush = nullptr;
    HIPC(hipMalloc(&flush, fl));
    std::vector<hipEvent_t> ev(2 * (size_t)reps);
    for (auto& e : ev) HIPC(hipEventCreate(&e));
    jx();  // warm-up
    for (int i = 0; i < reps; ++i) {
      HIPC(hipMemsetAsync(flush, i & 0xff, fl, c->stream));
      hipLaunchKernelGGL(k_read_sweep, dim3(1024), dim3(kBlock), 0, c->stream, static_cast<const double*>(flush),
                         (int64_t)(fl / sizeof(double)), c->partials);
      HIPC(hipEventRecord(ev[2 * i], c->stream));
      jx();
      HIPC(hipEventRecord(ev[2 * i + 1], c->stream));
    }
    HIPC(hipEventSynchronize(ev.back()));
    std::vector<double> t((size_t)reps);
    for (int i = 0; i < reps; ++i) {
      float f = 0.f;
      HIPC(hipEventElapsedTime(&f, ev[2 * i], ev[2 * i + 1]));
      t[(size_t)i] = f;
    }
    for (auto& e : ev) hipEventDestroy(e);
    HIPC(hipFree(flush));
    std::sort(t.begin(), t.end());
    *ms = (reps & 1) ? t[(size_t)reps / 2] : 0.5 * (t[(size_t)reps / 2 - 1] + t[(size_t)reps / 2]);
    return TV_OK;
  }
  if (int e = one()) return e;  // warm-up
  HIPC(hipEventRecord(c->ev0, c->stream));
  for (int i = 0; i < reps; ++i)
    if (int e = one()) return e;
  HIPC(hipEventRecord(c->ev1, c->stream));
  HIPC(hipEventSynchronize(c->ev1));
  float t = 0.f;
  HIPC(hipEventElapsedTime(&t, c->ev0, c->ev1));
  *ms = (double)t / reps;
  return TV_OK;
}


int tv_kernel_timing(void* ctx, int on) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c) return TV_ERR_ARG;
  hipSetDevice(c->device);
  for (int k = 0; k < 2; ++k)
    if (!c->vev[k]) HIPC(hipEventCreate(&c->vev[k]));
  if (!c->d_ts) {
    int khz = 0;
    HIPC(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device));
    if (khz <= 0) return c->fail(TV_ERR_HIP, "tv_kernel_timing: no device wall clock rate");
    c->ts_khz = (double)khz;
    HIPC(hipMalloc(&c->d_ts, (size_t)4 * kTsCap * sizeof(uint64_t)));
  }
  c->ts_pending.clear();
  c->ts_next = kTsCap;  // zeroes the stamps
  if (int e = ts_flush(c)) return e;
  if (int e = visco_timing_flush(c)) return e;  // a pending visco pair belongs to the old window
  c->ktime = on > 0;
  c->kstride = on > 1 ? on : 1;
  for (int k = 0; k < 3; ++k) {
    c->ksum[k] = 0.0;
    c->kcnt[k] = 0;
  }
  return TV_OK;
}


int tv_kernel_stats(void* ctx, int kernel, double* ms_avg, int64_t* launches) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c || !ms_avg) return TV_ERR_ARG;
  const int k = (kernel == 3) ? 0 : (kernel == 4) ? 1 : (kernel == 1) ? 2 : -1;
  if (k < 0) return c->fail(TV_ERR_ARG, "tv_kernel_stats: kernel 3 (fused matvec), 4 (PCG update) or 1 (visco)");
  hipSetDevice(c->device);
  if (int e = ts_flush(c)) return e;
  if (int e = visco_timing_flush(c)) return e;
  *ms_avg = c->kcnt[k] ? c->ksum[k] / (double)c->kcnt[k] : 0.0;
  if (launches) *launches = c->kcnt[k];
  return TV_OK;
}


int tv_pcg_variant(void* ctx, int* variant) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c || !variant) return TV_ERR_ARG;
  *variant = (c->cgs || c->mg_cgs) ? TV_PCG_SINGLE_REDUCTION : TV_PCG_KSPCG;
  return TV_OK;
}


int tv_last_stats(void* ctx, int* newton_its, int* krylov_its, double* dx_norm) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c) return TV_ERR_ARG;
  if (newton_its) *newton_its = c->last_newton;
  if (krylov_its) *krylov_its = c->last_krylov;
  if (dx_norm) *dx_norm = c->last_dx;
  return TV_OK;
}


int tv_last_converged(void* ctx, int* converged) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c || !converged) return TV_ERR_ARG;
  *converged = c->last_conv;
  return TV_OK;
}

}  // extern "C"
