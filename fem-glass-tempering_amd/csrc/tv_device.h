// Device-side helpers shared by the kernels of libtvfem.so: wave / block
// reductions, the last-arriving-workgroup hand-off (agent-scope release /
// acquire, MI355X_MICROARCH.md "Workgroup dispatch ... visibility"), and the
// scalar logic of PETSc KSPCG + KSPConvergedDefault (preconditioned norm).
#pragma once
#include "tv_internal.h"

namespace tv {

__device__ __forceinline__ double shr1(double v) {  // lane l <- lane l-1
  int lo = __double2loint(v), hi = __double2hiint(v);
  lo = __builtin_amdgcn_update_dpp(0, lo, 0x138, 0xF, 0xF, false);
  hi = __builtin_amdgcn_update_dpp(0, hi, 0x138, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double shl1(double v) {  // lane l <- lane l+1
  int lo = __double2loint(v), hi = __double2hiint(v);
  lo = __builtin_amdgcn_update_dpp(0, lo, 0x130, 0xF, 0xF, false);
  hi = __builtin_amdgcn_update_dpp(0, hi, 0x130, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

// A read-only table entry through the constant address space: a wave-uniform
// index becomes a scalar load (counted by lgkmcnt, so waiting for it does not
// wait for the vector loads in flight -- vmcnt counts in order)
template <class T>
__device__ __forceinline__ T kld(const T* p, int i) {
  return ((const __attribute__((address_space(4))) T*)p)[i];
}

// Blocks are dispatched round-robin over the 8 XCDs; remap so that each XCD
// gets a contiguous range of tile ids (bijective for any grid size), keeping
// the halo rows / columns shared by neighbouring tiles in one L2.
__device__ __forceinline__ int xcd_remap(int b, int nb) {
  const int q = nb >> 3, r = nb & 7, x = b & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}

__device__ __forceinline__ double wave_sum64(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Arrival protocol of the in-kernel reduction tail.  Every workgroup stores its
// partial record(s) WRITE-THROUGH (store_partial: sc1 / agent-scope atomic
// store), drains them (s_waitcnt vmcnt(0) in every wave, then a workgroup
// barrier), and one lane takes a ticket (relaxed agent-scope fetch_add).  The
// workgroup that draws the last ticket reads every record with sc1 loads
// (load_partial), so no agent release / acquire fence (buffer_wbl2 /
// buffer_inv) is needed (MI355X_MICROARCH.md "Valid forms", table row 1).
// The counter is re-armed (0) by the last workgroup.
__device__ __forceinline__ void store_partial(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double load_partial(const double* p) {
  return __hip_atomic_load(const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ bool last_block_arrived(unsigned* counter, unsigned nblocks) {
  __shared__ int amlast;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    amlast = (t == nblocks - 1) ? 1 : 0;
    if (amlast) __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  return amlast != 0;
}

// Fixed-order reduction of the records first, first + stride, ... (< n) of
// width W (<= 3) by one workgroup; the result is in sums[] of thread 0.
template <int W>
__device__ __forceinline__ void block_reduce_records(const double* partials, int first, int stride, int n,
                                                     double (&sums)[3]) {
  __shared__ double red[3][16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double acc[W];
#pragma unroll
  for (int w = 0; w < W; ++w) acc[w] = 0.0;
  // U records per thread in flight at once (the loads are independent; a
  // one-record loop would serialise n / blockDim latencies), summed in a
  // fixed order so the result stays bitwise reproducible.
  constexpr int U = 8;
  const int cnt = (n > first) ? (n - first + stride - 1) / stride : 0;
  for (int base = threadIdx.x; base < cnt; base += blockDim.x * U) {
    double v[U][W];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = base + u * (int)blockDim.x;
      const int64_t t = (int64_t)first + (int64_t)k * stride;
#pragma unroll
      for (int w = 0; w < W; ++w) v[u][w] = (k < cnt) ? load_partial(&partials[t * W + w]) : 0.0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int w = 0; w < W; ++w) acc[w] += v[u][w];
  }
#pragma unroll
  for (int w = 0; w < W; ++w) {
    const double s = wave_sum64(acc[w]);
    if (lane == 0) red[w][wave] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int nw = blockDim.x >> 6;
#pragma unroll
    for (int w = 0; w < W; ++w) {
      double s = 0.0;
      for (int q = 0; q < nw; ++q) s += red[w][q];
      sums[w] = s;
    }
  }
}

// ---- PETSc KSPSolve_CG + KSPConvergedDefault scalar logic -------------------
__device__ __forceinline__ void logic_init(PcgState* st, const double* sums) {
  const double dp = sqrt(sums[0]);
  st->dp = dp;
  st->rnorm0 = dp;
  st->ttol = fmax(st->rtol * dp, st->atol);
  st->it = 0;
  st->done = 0;
  st->reason = R_RUNNING;
  if (!isfinite(dp)) { st->done = 1; st->reason = R_DIV_NANINF; return; }
  if (dp <= st->ttol) { st->done = 1; st->reason = (dp <= st->atol) ? R_CONV_ATOL : R_CONV_RTOL; return; }
  st->beta = sums[1];
  st->betaold = 1.0;
  if (st->beta == 0.0) { st->done = 1; st->reason = R_CONV_ATOL; }
}

__device__ __forceinline__ void logic_dpi(PcgState* st, const double* sums) {
  if (st->done) return;
  const double dpi = sums[0];
  if (!isfinite(dpi)) { st->done = 1; st->reason = R_DIV_NANINF; return; }
  const double dpiold = st->dpiold;
  st->betaold = st->beta;
  if (dpi == 0.0 || (!st->relaxed && st->it > 0 && ((dpi > 0.0) != (dpiold > 0.0)))) {
    st->done = 1; st->reason = R_DIV_INDEF_MAT; return;
  }
  st->dpi = dpi;
  st->dpiold = dpi;
  st->a_prev = st->a;
  st->a = st->beta / dpi;
}

__device__ __forceinline__ void logic_update(PcgState* st, const double* sums) {
  if (st->done) return;
  const double dp = sqrt(sums[0]);
  st->it += 1;
  st->dp = dp;
  if (!isfinite(dp)) { st->done = 1; st->reason = R_DIV_NANINF; return; }
  if (dp <= st->ttol) { st->done = 1; st->reason = (dp <= st->atol) ? R_CONV_ATOL : R_CONV_RTOL; return; }
  if (dp >= st->dtol * st->rnorm0) { st->done = 1; st->reason = R_DIV_DTOL; return; }
  if (st->it >= st->max_it) { st->done = 1; st->reason = R_DIV_ITS; return; }
  const double beta = sums[1];
  if (beta == 0.0) { st->done = 1; st->reason = R_CONV_ATOL; return; }
  if (!st->relaxed && beta * st->betaold < 0.0) { st->done = 1; st->reason = R_DIV_INDEF_PC; return; }
  st->beta = beta;
}

// ---- the same logic for the single-reduction form (k_cgs_march) -------------
// sums = (gamma_i, delta_i, nu_i) = ((r_i, z_i), (z_i, J z_i), (z_i, z_i)).
// Iteration 0: PETSc's first pass up to alpha (dp test on ||z_0||, beta =
// (z, r) == 0 test, dpi = (p, A p) with p = z_0: delta_0).
__device__ __forceinline__ void logic_cgs_init(PcgState* st, const double* s) {
  const double dp = sqrt(s[2]);
  st->dp = dp;
  st->rnorm0 = dp;
  st->ttol = fmax(st->rtol * dp, st->atol);
  st->it = 0;
  st->done = 0;
  st->reason = R_RUNNING;
  if (!isfinite(dp)) { st->done = 1; st->reason = R_DIV_NANINF; return; }
  if (dp <= st->ttol) { st->done = 1; st->reason = (dp <= st->atol) ? R_CONV_ATOL : R_CONV_RTOL; return; }
  const double gamma = s[0];
  if (gamma == 0.0) { st->done = 1; st->reason = R_CONV_ATOL; return; }
  const double dpi = s[1];
  if (!isfinite(dpi)) { st->done = 1; st->reason = R_DIV_NANINF; return; }
  if (dpi == 0.0) { st->done = 1; st->reason = R_DIV_INDEF_MAT; return; }
  st->gamma = gamma;
  st->eta = dpi;
  st->beta = 0.0;
  st->a = gamma / dpi;
}

// Iteration i >= 1: the tests of logic_update on ||z_i|| and gamma_i, then
// beta_i = gamma_i / gamma_{i-1}, PETSc's dpi as eta_i = delta_i - beta_i
// gamma_i / alpha_{i-1} (= (p_i, A p_i) in exact arithmetic) with the tests of
// logic_dpi, alpha_i = gamma_i / eta_i.
__device__ __forceinline__ void logic_cgs(PcgState* st, const double* s) {
  if (st->done) return;
  const double dp = sqrt(s[2]);
  st->it += 1;
  st->dp = dp;
  if (!isfinite(dp)) { st->done = 1; st->reason = R_DIV_NANINF; return; }
  if (dp <= st->ttol) { st->done = 1; st->reason = (dp <= st->atol) ? R_CONV_ATOL : R_CONV_RTOL; return; }
  if (dp >= st->dtol * st->rnorm0) { st->done = 1; st->reason = R_DIV_DTOL; return; }
  if (st->it >= st->max_it) { st->done = 1; st->reason = R_DIV_ITS; return; }
  const double gamma = s[0];
  if (gamma == 0.0) { st->done = 1; st->reason = R_CONV_ATOL; return; }
  if (!st->relaxed && gamma * st->gamma < 0.0) { st->done = 1; st->reason = R_DIV_INDEF_PC; return; }
  const double beta = gamma / st->gamma;
  const double eta = s[1] - beta * gamma / st->a;
  if (!isfinite(eta)) { st->done = 1; st->reason = R_DIV_NANINF; return; }
  if (eta == 0.0 || (!st->relaxed && ((eta > 0.0) != (st->eta > 0.0)))) {
    st->done = 1;
    st->reason = R_DIV_INDEF_MAT;
    return;
  }
  st->beta = beta;
  st->gamma = gamma;
  st->eta = eta;
  st->a = gamma / eta;
}

// kinds 6 / 7: the single-reduction logic (5 / 4) on sums laid out as the
// multigrid form writes them -- (z.z, z.r) by the V-cycle's post-smoothing
// tail, then (z, A z) by the matvec's: (nu, gamma, delta)
__device__ __forceinline__ void apply_logic(PcgState* st, const double* sums, int kind) {
  if (kind == 1) logic_init(st, sums);
  else if (kind == 2) logic_dpi(st, sums);
  else if (kind == 3) logic_update(st, sums);
  else if (kind == 4) logic_cgs_init(st, sums);
  else if (kind == 5) logic_cgs(st, sums);
  else if (kind >= 6) {
    const double s[3] = {sums[1], sums[2], sums[0]};
    if (kind == 7) logic_cgs_init(st, s);
    else logic_cgs(st, s);
  }
}

// Lagged scalar logic (multi-rank): the state after the previous all-reduce,
// formed identically in every workgroup from *st and the all-reduced sums
// (lag != nullptr; logic `kind`).  The launch's tail workgroup forms it once
// more and commits it -- every workgroup has read *st by then, and nothing
// else writes *st or the sums before -- or, when it ends the solve, workgroup
// 0 commits it (commit_done) and every workgroup exits: a workgroup that reads
// the committed state concludes `done` as well.  (Forming it again in the tail
// keeps the ~30-dword state out of the kernel's registers.)
__device__ __forceinline__ PcgState lagged_state(const PcgState* st, const double* lag, int kind) {
  PcgState s = *st;
  if (lag != nullptr) apply_logic(&s, lag, kind);
  return s;
}
// logic_update's outcome on lagged sums as the fused matvec needs it (done,
// beta; betaold is unchanged by it), branch-free so that the march's first
// loads are not held behind the state: the same decisions as logic_update
__device__ __forceinline__ void lag_update_lean(const PcgState* st, const double* lag, int& done, double& beta) {
  const double dp = sqrt(lag[0]);
  const double b = lag[1];
  const bool stop = (st->done != 0) | !isfinite(dp) | (dp <= st->ttol) | (dp >= st->dtol * st->rnorm0) |
                    (st->it + 1 >= st->max_it) | (b == 0.0) | (!st->relaxed & (b * st->betaold < 0.0));
  done = stop ? 1 : 0;
  beta = stop ? st->beta : b;
}
__device__ __forceinline__ void commit_done(PcgState* st, const PcgState& s) {
  if (blockIdx.x == 0 && threadIdx.x == 0 && !st->done) *st = s;
}

// Tail of a kernel that produced one partial record (width W) per workgroup:
// the last workgroup to arrive reduces all n records in a fixed order into
// rt.out and (kind > 0) runs the PCG logic on the sums.  Measured alternative,
// not kept: a two-level tail with 8 shard counters (blockIdx % 8) and a top
// counter, against the ~12 ns per arrival that serialise on one counter
// (MI355X_MICROARCH.md price list "fanin"): 1-2 us SLOWER per launch at 0.1M,
// 1M and 8M nodes (the arrivals are spread out by the march's own skew; the
// extra hop is not).  Counters: rt.counter[0].
// rt.lag != nullptr: the launch's lagged state (lagged_state, formed from the
// sums before they are overwritten) is committed instead of running logic
// rt.kind on this launch's sums.
__device__ __forceinline__ void commit_lagged(const RedTail& rt) {
  const PcgState s = lagged_state(rt.st, rt.lag, rt.lag_kind);
  *rt.st = s;
}
template <int W>
__device__ __forceinline__ void fused_reduce_tail(const RedTail& rt, int n) {
  if (rt.counter == nullptr) return;
  if (!last_block_arrived(rt.counter, gridDim.x)) return;
  double sums[3] = {0.0, 0.0, 0.0};
  block_reduce_records<W>(rt.partials, 0, 1, n, sums);
  if (threadIdx.x == 0) {
    if (rt.lag != nullptr) commit_lagged(rt);  // reads rt.lag (== rt.out) first
    for (int w = 0; w < W; ++w) rt.out[w] = sums[w];
    if (rt.lag == nullptr) apply_logic(rt.st, sums, rt.kind);
    if (rt.ts) rt.ts[1] = __builtin_amdgcn_s_memrealtime();
  }
}

// Tail of the single-reduction iteration (records of width 3).  lag != nullptr
// (multi-rank, lagged logic): the sums are only reduced (RCCL all-reduces them
// next) and the tail workgroup commits the state this launch formed from the
// previous sums -- every workgroup has read the old state by the time the last
// one arrives.
__device__ __forceinline__ void cgs_tail(const RedTail& rt, int n, PcgState* st, const PcgState* lag) {
  if (rt.counter == nullptr) return;
  if (!last_block_arrived(rt.counter, gridDim.x)) return;
  double sums[3] = {0.0, 0.0, 0.0};
  block_reduce_records<3>(rt.partials, 0, 1, n, sums);
  if (threadIdx.x == 0) {
    for (int w = 0; w < 3; ++w) rt.out[w] = sums[w];
    if (lag) *st = *lag;
    else apply_logic(rt.st, sums, rt.kind);
    if (rt.ts) rt.ts[1] = __builtin_amdgcn_s_memrealtime();
  }
}

// Robin facet terms of node t (local index t + t_off) left out of w by the
// fused CG matvec (marching path); 0 off the physical boundary faces
__device__ __forceinline__ double face_terms(const FaceAdd& fa, int64_t t) {
  const int nd = (int)(t + fa.t_off);
  const int plane = fa.n0 * fa.n1;
  int k = (int)((double)nd * fa.inv_plane);
  k -= (k * plane > nd) ? 1 : 0;
  k += ((k + 1) * plane <= nd) ? 1 : 0;
  const int rem = nd - k * plane;
  int j = (int)((double)rem * fa.inv_n0);
  j -= (j * fa.n0 > rem) ? 1 : 0;
  j += ((j + 1) * fa.n0 <= rem) ? 1 : 0;
  const int i = rem - j * fa.n0;
  double add = 0.0;
  if (i == 0 && fa.ff[0]) add += fa.ff[0][j + fa.n1 * k];
  if (i == fa.n0 - 1 && fa.ff[1]) add += fa.ff[1][j + fa.n1 * k];
  if (j == 0 && fa.ff[2]) add += fa.ff[2][i + fa.n0 * k];
  if (j == fa.n1 - 1 && fa.ff[3]) add += fa.ff[3][i + fa.n0 * k];
  if (k == 0 && fa.ff[4]) add += fa.ff[4][i + fa.n0 * j];
  if (k == fa.n2 - 1 && fa.ff[5]) add += fa.ff[5][i + fa.n0 * j];
  return add;
}

// face_terms with every load issued unconditionally (for the latency-bound
// coarse-level kernels: a load under the node's face test made the wave wait
// for it at once, after everything in flight).  One buffer resource over the
// level's face buffer (one allocation, the faces in order, CgGrid::ffbuf), an
// out-of-range offset where the node is on neither face of a pair; the sum in
// face_terms' order.
struct FaceRsrc {
  __amdgpu_buffer_rsrc_t r;
  int64_t d[6];  // element offset of face g from the buffer's base
};
__device__ __forceinline__ FaceRsrc face_rsrc(const FaceAdd& fa) {
  FaceRsrc fr{};
  const double* fb = nullptr;
  int64_t fend = 0;
#pragma unroll
  for (int g = 0; g < 6; ++g)
    if (fa.ff[g] != nullptr) {
      if (fb == nullptr) fb = fa.ff[g];
      const int64_t sz = (g >> 1) == 0 ? (int64_t)fa.n1 * fa.n2
                                        : ((g >> 1) == 1 ? (int64_t)fa.n0 * fa.n2 : (int64_t)fa.n0 * fa.n1);
      fend = (int64_t)(fa.ff[g] - fb) + sz;
    }
#pragma unroll
  for (int g = 0; g < 6; ++g) fr.d[g] = fa.ff[g] ? (int64_t)(fa.ff[g] - fb) : 0;
  const uint64_t a = (uint64_t)fb;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  void* q = (void*)(((uint64_t)hi << 32) | lo);
  fr.r = __builtin_amdgcn_make_buffer_rsrc(q, (short)0, (int)__builtin_amdgcn_readfirstlane((uint32_t)(fb ? fend * 8 : 0)),
                                           0x00020000);
  return fr;
}
__device__ __forceinline__ double face_terms_nb(const FaceAdd& fa, const FaceRsrc& fr, int64_t t) {
  const int nd = (int)(t + fa.t_off);
  const int plane = fa.n0 * fa.n1;
  int k = (int)((double)nd * fa.inv_plane);
  k -= (k * plane > nd) ? 1 : 0;
  k += ((k + 1) * plane <= nd) ? 1 : 0;
  const int rem = nd - k * plane;
  int j = (int)((double)rem * fa.inv_n0);
  j -= (j * fa.n0 > rem) ? 1 : 0;
  j += ((j + 1) * fa.n0 <= rem) ? 1 : 0;
  const int i = rem - j * fa.n0;
  const bool x0 = i == 0 && fa.ff[0], x1 = i == fa.n0 - 1 && fa.ff[1];
  const bool y0 = j == 0 && fa.ff[2], y1 = j == fa.n1 - 1 && fa.ff[3];
  const bool z0 = k == 0 && fa.ff[4], z1 = k == fa.n2 - 1 && fa.ff[5];
  constexpr uint32_t kOut = 0x40000000u;
  const uint32_t ox = (x0 || x1) ? (uint32_t)((x0 ? fr.d[0] : fr.d[1]) + j + (int64_t)fa.n1 * k) * 8u : kOut;
  const uint32_t oy = (y0 || y1) ? (uint32_t)((y0 ? fr.d[2] : fr.d[3]) + i + (int64_t)fa.n0 * k) * 8u : kOut;
  const uint32_t oz = (z0 || z1) ? (uint32_t)((z0 ? fr.d[4] : fr.d[5]) + i + (int64_t)fa.n0 * j) * 8u : kOut;
  const double fx = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(fr.r, (int)ox, 0, 0));
  const double fy = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(fr.r, (int)oy, 0, 0));
  const double fz = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(fr.r, (int)oz, 0, 0));
  return (fx + fy) + fz;
}

// face_at with every load issued unconditionally (FaceRsrc, as face_terms_nb)
__device__ __forceinline__ double face_at_nb(const FaceAdd& fa, const FaceRsrc& fr, int i, int j, int k) {
  const bool x0 = i == 0 && fa.ff[0], x1 = i == fa.n0 - 1 && fa.ff[1];
  const bool y0 = j == 0 && fa.ff[2], y1 = j == fa.n1 - 1 && fa.ff[3];
  const bool z0 = k == 0 && fa.ff[4], z1 = k == fa.n2 - 1 && fa.ff[5];
  constexpr uint32_t kOut = 0x40000000u;
  const uint32_t ox = (x0 || x1) ? (uint32_t)((x0 ? fr.d[0] : fr.d[1]) + j + (int64_t)fa.n1 * k) * 8u : kOut;
  const uint32_t oy = (y0 || y1) ? (uint32_t)((y0 ? fr.d[2] : fr.d[3]) + i + (int64_t)fa.n0 * k) * 8u : kOut;
  const uint32_t oz = (z0 || z1) ? (uint32_t)((z0 ? fr.d[4] : fr.d[5]) + i + (int64_t)fa.n0 * j) * 8u : kOut;
  const double fx = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(fr.r, (int)ox, 0, 0));
  const double fy = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(fr.r, (int)oy, 0, 0));
  const double fz = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(fr.r, (int)oz, 0, 0));
  return (fx + fy) + fz;
}

// the same at local node (i, j, k) (coordinates known)
__device__ __forceinline__ double face_at(const FaceAdd& fa, int i, int j, int k) {
  double add = 0.0;
  if (i == 0 && fa.ff[0]) add += fa.ff[0][j + fa.n1 * k];
  if (i == fa.n0 - 1 && fa.ff[1]) add += fa.ff[1][j + fa.n1 * k];
  if (j == 0 && fa.ff[2]) add += fa.ff[2][i + fa.n0 * k];
  if (j == fa.n1 - 1 && fa.ff[3]) add += fa.ff[3][i + fa.n0 * k];
  if (k == 0 && fa.ff[4]) add += fa.ff[4][i + fa.n0 * j];
  if (k == fa.n2 - 1 && fa.ff[5]) add += fa.ff[5][i + fa.n0 * j];
  return add;
}

// Start stamp of a launch with a timed reduction tail: workgroup 0 is the
// first one the dispatcher places, so its entry time is the launch's start.
__device__ __forceinline__ void stamp_start(const RedTail& rt) {
  if (rt.ts && blockIdx.x == 0 && threadIdx.x == 0) rt.ts[0] = __builtin_amdgcn_s_memrealtime();
}

}  // namespace tv
