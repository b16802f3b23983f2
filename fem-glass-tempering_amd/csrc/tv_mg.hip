// Geometric multigrid on the box hierarchy: grid-transfer and smoothing
// kernels of the V-cycle preconditioner (gfx950).
//
// Replaces, for 3D CG1 rectilinear meshes, the algebraic multigrid the
// reference configures for its Krylov solve (PCGAMG, ThermoViscoProblem.py:
// 343-346).  The hierarchy is the box itself, every other node kept along each
// axis (plus the last node when the cell count is odd, so the coarse nodes are
// always a subset of the fine ones: P is exact linear interpolation, R = P^T);
// the coarse operators are the same matrix-free tensor-product Jacobian on the
// coarse grid (tv_cg.hip), with T injected.  Smoother: damped Jacobi, omega =
// 2 / (1.1 b) with b the Gershgorin bound of D^-1 J (exact row sums of the
// 27-point stencil), the same polynomial before and after the coarse
// correction, so the V-cycle is a fixed symmetric positive definite operator
// (CG stays CG).
//
// Every kernel exits at once when the solve has converged (st->done), so the
// V-cycles queued behind the converged iteration cost a launch each.
// Bytes (algorithmic, per node of the level): restriction 16 (r, w of the fine
// level) + 8 / 8 (coarse write), prolongation 16 (+ coarse reads, cached),
// Jacobi step 24 / 40.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "tv_stencil.h"

namespace tv {
namespace {

// One thread per output node (flat index over the owned planes, 32-bit decode).
// b_c(I) = sum over the 3 x 3 x 3 fine nodes f of w(f, I) (b_f - w_f)(f)
template <bool MASK>
__global__ __launch_bounds__(kBlock) void k_mg_restrict(MgXfer x, const PcgState* __restrict__ st,
                                                        const double* __restrict__ bf,
                                                        const double* __restrict__ wf,
                                                        const double* __restrict__ mask, double* __restrict__ bc,
                                                        const double* __restrict__ dinv_c, double omega_c,
                                                        double* __restrict__ xc) {
  if (st != nullptr && st->done) return;
  const int plane = x.cn[0] * x.cn[1];
  const int n = plane * (x.c_ke - x.c_kb);
  const int fpl = x.fn[0] * x.fn[1];
  // a contiguous range of output nodes per block, contiguous block ranges per
  // XCD (xcd_remap): the fine rows a range gathers stay in one L2
  const int per = (n + (int)gridDim.x - 1) / (int)gridDim.x;
  const int t0 = xcd_remap(blockIdx.x, gridDim.x) * per, t1 = min(n, t0 + per);
  int k = (t0 + (int)threadIdx.x) / plane, j, i;
  {
    const int rem = t0 + (int)threadIdx.x - k * plane;
    j = rem / x.cn[0];
    i = rem - j * x.cn[0];
  }
  k += x.c_kb;
  for (int t = t0 + (int)threadIdx.x; t < t1; t += kBlock, i += kBlock) {
    while (i >= x.cn[0]) {  // advance (i, j, k) by kBlock nodes
      i -= x.cn[0];
      if (++j == x.cn[1]) {
        j = 0;
        ++k;
      }
    }
    int fi[3], fj[3], fk[3];
    rmap(x, 0, i, fi[0], fi[1], fi[2]);
    rmap(x, 1, j, fj[0], fj[1], fj[2]);
    rmap(x, 2, k, fk[0], fk[1], fk[2]);
    double wi[3], wj[3], wk[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      wi[q] = x.rw[0][3 * i + q];
      wj[q] = x.rw[1][3 * j + q];
      wk[q] = x.rw[2][3 * k + q];
    }
    double acc = 0.0;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      double pl = 0.0;
#pragma unroll
      for (int b = 0; b < 3; ++b) {
        const int base = fj[b] * x.fn[0] + fpl * fk[c];
        double row = 0.0;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          const int f = base + fi[a];
          double r = bf[f] - wf[f];
          if (MASK && mask[f] == 0.0) r = 0.0;
          row += wi[a] * r;
        }
        pl += wj[b] * row;
      }
      acc += wk[c] * pl;
    }
    const int o = t + plane * x.c_kb;
    bc[o] = acc;
    if (xc != nullptr) xc[o] = omega_c * dinv_c[o] * acc;  // the coarse pre-smoothing step from 0
  }
}

// x_f(f) += sum over the 2 x 2 x 2 coarse nodes I of w(f, I) x_c(I).  A block
// owns kPU x kBlock consecutive fine nodes; a thread decodes its kPU nodes
// first and issues all their gathers before the first FMA (one node per
// round left each wave waiting on its load chain: 54 us at 8.2M nodes).
constexpr int kPU = 2;
__global__ __launch_bounds__(kBlock) void k_mg_prolong(MgXfer x, const PcgState* __restrict__ st,
                                                       double* __restrict__ xf, const double* __restrict__ xc,
                                                       const double* __restrict__ mask) {
  if (st != nullptr && st->done) return;
  const int plane = x.fn[0] * x.fn[1];
  const int n = plane * (x.f_ke - x.f_kb);
  const int cpl = x.cn[0] * x.cn[1];
  const int t0 = xcd_remap(blockIdx.x, gridDim.x) * (kPU * kBlock) + (int)threadIdx.x;
  int k = t0 / plane, j, i;
  {
    const int rem = t0 - k * plane;
    j = rem / x.fn[0];
    i = rem - j * x.fn[0];
  }
  k += x.f_kb;
  int f[kPU], o[kPU][8];
  double w[kPU][6];
#pragma unroll
  for (int u = 0; u < kPU; ++u) {
    if (u > 0) {
      i += kBlock;
      while (i >= x.fn[0]) {
        i -= x.fn[0];
        if (++j == x.fn[1]) {
          j = 0;
          ++k;
        }
      }
    }
    const int t = t0 + u * kBlock;
    const bool ok = t < n;
    const int ii = ok ? i : 0, jj = ok ? j : 0, kk = ok ? k : x.f_kb;
    f[u] = ok ? t + plane * x.f_kb : -1;
    int ci[2], cj[2], ck[2];
    pmap(x, 0, ii, ci[0], ci[1]);
    pmap(x, 1, jj, cj[0], cj[1]);
    pmap(x, 2, kk, ck[0], ck[1]);
#pragma unroll
    for (int q = 0; q < 8; ++q) o[u][q] = ci[q & 1] + x.cn[0] * cj[(q >> 1) & 1] + cpl * ck[q >> 2];
    w[u][0] = x.pw[0][2 * ii]; w[u][1] = x.pw[0][2 * ii + 1];
    w[u][2] = x.pw[1][2 * jj]; w[u][3] = x.pw[1][2 * jj + 1];
    w[u][4] = x.pw[2][2 * kk]; w[u][5] = x.pw[2][2 * kk + 1];
  }
  double v[kPU][8], xo[kPU];
#pragma unroll
  for (int u = 0; u < kPU; ++u) {
#pragma unroll
    for (int q = 0; q < 8; ++q) v[u][q] = xc[o[u][q]];
    xo[u] = f[u] >= 0 ? xf[f[u]] : 0.0;
  }
#pragma unroll
  for (int u = 0; u < kPU; ++u) {
    if (f[u] < 0) continue;
    const double p0 = w[u][2] * (w[u][0] * v[u][0] + w[u][1] * v[u][1]) + w[u][3] * (w[u][0] * v[u][2] + w[u][1] * v[u][3]);
    const double p1 = w[u][2] * (w[u][0] * v[u][4] + w[u][1] * v[u][5]) + w[u][3] * (w[u][0] * v[u][6] + w[u][1] * v[u][7]);
    const double acc = w[u][4] * p0 + w[u][5] * p1;
    const bool off = mask != nullptr && mask[f[u]] == 0.0;
    xf[f[u]] = off ? 0.0 : xo[u] + acc;
  }
}

// ---- x-pair transfers --------------------------------------------------------
// A lane owns the fine pair (2I, 2I + 1) of coarse x node I and moves it with
// ONE 16-byte load / store (rows of an odd node count start 8-byte aligned:
// gfx950 buffer / global accesses need dword alignment only), so a wave's
// access is one contiguous 1 KB run per row instead of two 8-byte-strided
// ones (half the load instructions and half the L1 lines per fine node of the
// row-per-wave kernels above).  The x neighbour across the pair boundary comes
// from the adjacent lane (DPP wave shift); the segment's first (restriction)
// or last (prolongation) lane only loads it for its neighbour.
typedef double d2a8 __attribute__((ext_vector_type(2), aligned(8)));
constexpr int kPairSeg = kWave - 1;  // outputs per wave

__device__ __forceinline__ d2a8 ld_pair(const double* p) { return *reinterpret_cast<const d2a8*>(p); }
// a pair not read again: non-temporal (leaves the caches to the vectors that are)
__device__ __forceinline__ d2a8 ld_pair_nt(const double* p) { return __builtin_nontemporal_load(reinterpret_cast<const d2a8*>(p)); }

// the row-axis / plane-axis face terms of face_at (faces 2 .. 5), added to
// `add` in face_at's order
__device__ __forceinline__ double face_rows_add(const FaceAdd& fa, double add, int i, int j, int k) {
  if (j == 0 && fa.ff[2]) add += fa.ff[2][i + fa.n0 * k];
  if (j == fa.n1 - 1 && fa.ff[3]) add += fa.ff[3][i + fa.n0 * k];
  if (k == 0 && fa.ff[4]) add += fa.ff[4][i + fa.n0 * j];
  if (k == fa.n2 - 1 && fa.ff[5]) add += fa.ff[5][i + fa.n0 * j];
  return add;
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t xf_rsrc(const void* p, uint32_t bytes) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  void* q = (void*)(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(q, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
__device__ __forceinline__ double xf_ld1(__amdgpu_buffer_rsrc_t r, uint32_t voff) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, (int)voff, 0, 0));
}

// Restriction, one wave per (coarse row, 63-node x segment); lane l is coarse
// node I = 63 seg - 1 + l (lane 0 = the halo lane whose right fine node is
// lane 1's left neighbour).  A lane whose fine centre is the row's last node
// (even cell count, or the odd tail) loads that node alone; its right weight is 0.
// FACES: wf is a partial J x (k_cg_march without k_cg_addfaces); the facet
// terms of the face-workgroup faces (fa) are added here, on the boundary rows
// (wave-uniform test) and the two x-boundary lanes only -- one launch fewer per
// coarse level (bitwise the same r - (w + faces) as with k_cg_addfaces).  The
// x-face terms are loaded with the rows, unconditionally (an out-of-range
// offset off the x-boundary lanes): loaded under the lane test (face_at) they
// made every segment-0 / last-segment wave wait for all its loads nine times
template <bool MASK, bool FACES = false>
__global__ __launch_bounds__(kWave) void k_mg_restrict_pairs(MgXfer x, const PcgState* __restrict__ st,
                                                             const double* __restrict__ bf,
                                                             const double* __restrict__ wf,
                                                             const double* __restrict__ mask, double* __restrict__ bc,
                                                             const double* __restrict__ dinv_c, double omega_c,
                                                             double* __restrict__ xc, int nseg, FaceAdd fa) {
  if (st != nullptr && st->done) return;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int row = bid / nseg;
  const int seg = bid - row * nseg;
  const int J = row % x.cn[1], K = row / x.cn[1] + x.c_kb;
  const int lane = (int)threadIdx.x;
  const int cn = x.cn[0], nf = x.fn[0];
  const int I = seg * kPairSeg - 1 + lane;
  const bool ok = lane > 0 && I < cn;
  const int II = I < 0 ? 0 : (I < cn ? I : cn - 1);
  const int f1 = (II == cn - 1 && ((nf - 1) & 1)) ? nf - 1 : 2 * II;
  const bool pair = f1 + 1 < nf;
  const double wl = x.rw[0][3 * II], wr = x.rw[0][3 * II + 2];
  const int64_t fpl = (int64_t)nf * x.fn[1];
  const int64_t o = (int64_t)I + (int64_t)cn * (J + (int64_t)x.cn[1] * K);
  // the output's coarse diagonal first: its load overlaps the gathers below
  // (clamped address, no branch around the load)
  const double dcl = (xc != nullptr) ? dinv_c[(int64_t)II + (int64_t)cn * (J + (int64_t)x.cn[1] * K)] : 0.0;
  const double dci = ok ? dcl : 0.0;
  // fine rows / planes of the 3 x 3 gather: closed form along axis 1 (always a
  // whole axis) and, on a whole-box level, along axis 2 -- no table load ahead
  // of the gathers (a partitioned level's local axis-2 window keeps its table)
  int fjr[3], fkr[3];
  rmap(x, 1, J, fjr[0], fjr[1], fjr[2]);
  if (x.aligned) {
    rmap(x, 2, K, fkr[0], fkr[1], fkr[2]);
  } else {
#pragma unroll
    for (int c = 0; c < 3; ++c) fkr[c] = x.ri[2][3 * K + c];
  }
  // all 9 rows' loads first, then the arithmetic: loads under a per-lane
  // branch (the odd tail lane's single node) made every row wait for the one
  // before (vmcnt counts in order) -- 9 memory round trips per wave.  The tail
  // lane loads the pair ending at its node (always inside the row) and keeps .y
  d2a8 rv[9], wv[9], mv[9];
  int fjq[9], fkq[9];
  double dc[9], dr[9], wq[9];
  // FACES: this lane's x-face node -- the pair's .x at fine x 0 (face 0), its
  // .y at nf - 1 (face 1) or the odd tail lane's node nf - 1 (face 1); the two
  // x-face arrays through one resource (one allocation, CgGrid::ffbuf)
  const bool xlo = FACES && fa.ff[0] != nullptr && f1 == 0;
  const bool xhi = FACES && fa.ff[1] != nullptr && (pair ? f1 + 1 == nf - 1 : f1 == nf - 1);
  const double* fxb = fa.ff[0] ? fa.ff[0] : fa.ff[1];
  const int64_t dx1 = (fa.ff[0] && fa.ff[1]) ? (int64_t)(fa.ff[1] - fa.ff[0]) : 0;
  const __amdgpu_buffer_rsrc_t rfx =
      xf_rsrc(fxb, (FACES && fxb) ? (uint32_t)((dx1 + (int64_t)fa.n1 * fa.n2) * 8) : 0u);
  const uint32_t fxo = xhi ? (uint32_t)dx1 : 0u;
  // only the waves holding an x-face lane issue them (segment 0 and the last)
  const bool xwave = FACES && __ballot(xlo || xhi) != 0;  // wave-uniform
  double xfv[9];
#pragma unroll
  for (int q = 0; q < 9; ++q) {
    const int c = q / 3, b = q % 3;
    wq[q] = x.rw[2][3 * K + c] * x.rw[1][3 * J + b];
    fjq[q] = fjr[b];
    fkq[q] = fkr[c];
    const int64_t f = (int64_t)fjr[b] * nf + fpl * fkr[c] + f1;
    const int64_t fp = pair ? f : f - 1;
    rv[q] = ld_pair(bf + fp);
    wv[q] = (wf != nullptr) ? ld_pair_nt(wf + fp) : d2a8{0.0, 0.0};  // wf null: bf is the residual itself
    if (MASK) mv[q] = ld_pair(mask + fp);
    xfv[q] = 0.0;
  }
  if (xwave) {  // all nine issued back to back, no wait between them
#pragma unroll
    for (int q = 0; q < 9; ++q)
      xfv[q] = xf_ld1(rfx, (xlo || xhi) ? (fxo + (uint32_t)(fjr[q % 3] + fa.n1 * fkr[q / 3])) * 8u : 0x40000000u);
  }
#pragma unroll
  for (int q = 0; q < 9; ++q) {
    const int fj = fjq[q], fk = fkq[q];
    const bool rowface = FACES && ((fa.ff[2] && fj == 0) || (fa.ff[3] && fj == fa.n1 - 1) || (fa.ff[4] && fk == 0) ||
                                   (fa.ff[5] && fk == fa.n2 - 1));  // wave-uniform
    if (pair) {
      const d2a8 r = rv[q];
      d2a8 w = wv[q];
      if (FACES) {  // face_at's sums: the x face first, then faces 2 .. 5 (rare rows: loads under the branch)
        double ax = xlo ? xfv[q] : 0.0, ay = xhi ? xfv[q] : 0.0;
        if (rowface) {
          ax = face_rows_add(fa, ax, f1, fj, fk);
          ay = face_rows_add(fa, ay, f1 + 1, fj, fk);
        }
        if (rowface || f1 == 0) w.x += ax;
        if (rowface || f1 + 1 == nf - 1) w.y += ay;
      }
      dc[q] = r.x - w.x;
      dr[q] = r.y - w.y;
      if (MASK) {
        const d2a8 m = mv[q];
        if (m.x == 0.0) dc[q] = 0.0;
        if (m.y == 0.0) dr[q] = 0.0;
      }
    } else {
      double wt = wv[q].y;
      if (FACES) {  // the row's last node: an x-face node
        double add = xhi ? xfv[q] : 0.0;
        if (rowface) add = face_rows_add(fa, add, f1, fj, fk);
        wt += add;
      }
      double d = rv[q].y - wt;
      if (MASK && mv[q].y == 0.0) d = 0.0;
      dc[q] = dr[q] = d;
    }
  }
  double acc = 0.0;
#pragma unroll
  for (int q = 0; q < 9; ++q) {
    const double dl = shr1(dr[q]);  // lane - 1's right fine node = 2I - 1 (weight 0 at I = 0 and the odd tail)
    acc += wq[q] * ((wl * dl + dc[q]) + wr * dr[q]);
  }
  if (!ok) return;
  bc[o] = acc;
  if (xc != nullptr) xc[o] = omega_c * dci * acc;  // the coarse pre-smoothing step from 0
}

// Prolongation, one wave per (fine row, 63-pair segment); lane l owns the fine
// pair (2c, 2c + 1), c = 63 seg + l; lane 63 only loads coarse c for lane 62.
// Fine 2c is coarse c; fine 2c + 1 interpolates c and c + 1 (lane + 1), or is
// the odd tail (coarse c + 1 itself).
__global__ __launch_bounds__(kWave) void k_mg_prolong_pairs(MgXfer x, const PcgState* __restrict__ st,
                                                            double* __restrict__ xf, const double* __restrict__ xc,
                                                            const double* __restrict__ mask, int nseg) {
  if (st != nullptr && st->done) return;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int row = bid / nseg;
  const int seg = bid - row * nseg;
  const int j = row % x.fn[1], k = row / x.fn[1] + x.f_kb;
  const int nf = x.fn[0], cn = x.cn[0];
  const int lane = (int)threadIdx.x;
  const int c = seg * kPairSeg + lane;
  const int cc = c < cn ? c : cn - 1;
  const int i0 = 2 * c, i1 = 2 * c + 1;
  const bool has0 = lane < kPairSeg && i0 < nf, has1 = lane < kPairSeg && i1 < nf;
  const bool tail = i1 == nf - 1 && ((nf - 1) & 1);
  const int i1c = has1 ? i1 : 0;
  const double wl = x.pw[0][2 * i1c], wr = x.pw[0][2 * i1c + 1];
  const int64_t cpl = (int64_t)cn * x.cn[1];
  const int64_t f = (int64_t)i0 + (int64_t)nf * (j + (int64_t)x.fn[1] * k);
  double v[4], w[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int cz = q >> 1, b = q & 1;
    w[q] = x.pw[2][2 * k + cz] * x.pw[1][2 * j + b];
    v[q] = xc[cc + (int64_t)cn * x.pi[1][2 * j + b] + cpl * x.pi[2][2 * k + cz]];
  }
  d2a8 xo = {0.0, 0.0};
  if (has1) xo = ld_pair(xf + f);
  else if (has0) xo.x = xf[f];
  double a0 = 0.0, a1 = 0.0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const double vr = shl1(v[q]);  // coarse c + 1
    a0 += w[q] * v[q];
    a1 += w[q] * (tail ? vr : wl * v[q] + wr * vr);
  }
  if (!has0) return;
  if (has1) {
    d2a8 out = {xo.x + a0, xo.y + a1};
    if (mask != nullptr) {
      const d2a8 m = ld_pair(mask + f);
      if (m.x == 0.0) out.x = 0.0;
      if (m.y == 0.0) out.y = 0.0;
    }
    *reinterpret_cast<d2a8*>(xf + f) = out;
  } else {
    const bool off = mask != nullptr && mask[f] == 0.0;
    xf[f] = off ? 0.0 : xo.x + a0;
  }
}

// Prolongation by 2 x 2 blocks of fine rows (all three axes coarsened, one
// partition): fine rows (2jb + a, 2kb + c) interpolate only from the coarse
// rows (jb, jb + 1) x (kb, kb + 1) (the odd tail too), so a wave loads those
// four coarse x-runs once for four fine rows -- 4 coarse loads per 4 x 128 fine
// nodes instead of 16, and four 1 KB fine runs in flight per wave.
// SMOOTH: the coarse level's post-smoothing step, xc + omega dinv (b - (w +
// facet terms)), is formed on the fly from its operands (CoarsePost) instead
// of by a k_mg_jacobi launch that would write xc back (the prolongation is the
// smoothed xc's only reader)
template <bool SMOOTH>
__global__ __launch_bounds__(kWave) void k_mg_prolong_blk(MgXfer x, const PcgState* __restrict__ st,
                                                          double* __restrict__ xf, const double* __restrict__ xc,
                                                          const double* __restrict__ mask, int nseg, int nbj,
                                                          CoarsePost cp) {
  if (st != nullptr && st->done) return;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int blk = bid / nseg;
  const int seg = bid - blk * nseg;
  const int jb = blk % nbj, kb = blk / nbj;
  const int nf = x.fn[0], cn = x.cn[0];
  const int lane = (int)threadIdx.x;
  const int c = seg * kPairSeg + lane;
  const int cc = c < cn ? c : cn - 1;
  const int i0 = 2 * c, i1 = 2 * c + 1;
  const bool has0 = lane < kPairSeg && i0 < nf, has1 = lane < kPairSeg && i1 < nf;
  const bool tail = i1 == nf - 1 && ((nf - 1) & 1);
  const int i1c = has1 ? i1 : 0;
  const double wl = x.pw[0][2 * i1c], wr = x.pw[0][2 * i1c + 1];
  const int64_t cpl = (int64_t)cn * x.cn[1];
  const int jc1 = min(jb + 1, x.cn[1] - 1), kc1 = min(kb + 1, x.cn[2] - 1);
  // every load first, then the arithmetic (loads under per-lane branches, or
  // after a branchy face_at, made each wait for the ones before: vmcnt counts
  // in order): the four coarse x-runs (and the post-smoothing operands), then
  // the four fine rows' old values -- the lone-node lane at the row's odd end
  // loads the pair ending at its node, rows past the grid a clamped row (not
  // stored); the fine-row weights are wave-uniform scalar loads
  double v[4], cw[4], cd[4], cb[4];
  // SMOOTH: the coarse facet terms (face_at) with the operands -- one resource
  // over the coarse level's face buffer (one allocation, faces in order), an
  // out-of-range offset where a node is on no face of the pair; loaded under the
  // face tests they cost the waves that hold face nodes another round trip each
  const FaceAdd& fa = cp.fa;
  const double* fb = nullptr;
  int64_t fend = 0;
  if (SMOOTH) {
#pragma unroll
    for (int g = 0; g < 6; ++g)
      if (fa.ff[g] != nullptr) {
        if (fb == nullptr) fb = fa.ff[g];
        const int64_t sz = (g >> 1) == 0 ? (int64_t)fa.n1 * fa.n2 : ((g >> 1) == 1 ? (int64_t)fa.n0 * fa.n2 : (int64_t)fa.n0 * fa.n1);
        fend = (int64_t)(fa.ff[g] - fb) + sz;
      }
  }
  const __amdgpu_buffer_rsrc_t rfa = xf_rsrc(fb, SMOOTH && fb ? (uint32_t)(fend * 8) : 0u);
  // element offsets of the six faces (uniform; selected per lane below, never
  // indexed by a lane value: that puts the argument struct in memory)
  int64_t fd[6];
#pragma unroll
  for (int g = 0; g < 6; ++g) fd[g] = (SMOOTH && fa.ff[g]) ? (int64_t)(fa.ff[g] - fb) : 0;
  double fv[4][3];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int jcq = (q & 1) ? jc1 : jb, kcq = (q >> 1) ? kc1 : kb;
    const int64_t o = cc + (int64_t)cn * jcq + cpl * kcq;
    v[q] = xc[o];
    if (SMOOTH) {
      cw[q] = cp.w[o];
      cd[q] = cp.dinv[o];
      cb[q] = cp.b[o];
    }
    fv[q][0] = fv[q][1] = fv[q][2] = 0.0;
  }
  // only the waves holding a face node issue the face loads (all twelve back to
  // back): an x-boundary lane, or a boundary coarse row / plane (wave-uniform)
  const bool fwave = SMOOTH && (__ballot(cc == 0 || cc == cn - 1) != 0 || jb == 0 || jc1 == fa.n1 - 1 || kb == 0 ||
                                kc1 == fa.n2 - 1);
  if (fwave) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int jcq = (q & 1) ? jc1 : jb, kcq = (q >> 1) ? kc1 : kb;
      const bool x0 = cc == 0 && fa.ff[0], x1 = cc == fa.n0 - 1 && fa.ff[1];
      const bool y0 = jcq == 0 && fa.ff[2], y1 = jcq == fa.n1 - 1 && fa.ff[3];
      const bool z0 = kcq == 0 && fa.ff[4], z1 = kcq == fa.n2 - 1 && fa.ff[5];
      const int64_t ex = (x0 ? fd[0] : fd[1]) + jcq + (int64_t)fa.n1 * kcq;
      const int64_t ey = (y0 ? fd[2] : fd[3]) + cc + (int64_t)fa.n0 * kcq;
      const int64_t ez = (z0 ? fd[4] : fd[5]) + cc + (int64_t)fa.n0 * jcq;
      fv[q][0] = xf_ld1(rfa, (x0 || x1) ? (uint32_t)ex * 8u : 0x40000000u);
      fv[q][1] = xf_ld1(rfa, (y0 || y1) ? (uint32_t)ey * 8u : 0x40000000u);
      fv[q][2] = xf_ld1(rfa, (z0 || z1) ? (uint32_t)ez * 8u : 0x40000000u);
    }
  }
  bool rj[2], rk[2];
  int64_t f[4];
  d2a8 xo[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int a = r & 1, b = r >> 1;
    const int jr = min(2 * jb + a, x.fn[1] - 1), kr = min(2 * kb + b, x.f_ke - 1);
    f[r] = (int64_t)i0 + (int64_t)nf * (jr + (int64_t)x.fn[1] * kr);
    const int64_t fp = (int64_t)(has1 ? i0 : nf - 2) + (int64_t)nf * (jr + (int64_t)x.fn[1] * kr);
    const d2a8 t = ld_pair(xf + fp);
    xo[r] = d2a8{has1 ? t.x : (has0 ? t.y : 0.0), has1 ? t.y : 0.0};
  }
  if (SMOOTH) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int jcq = (q & 1) ? jc1 : jb, kcq = (q >> 1) ? kc1 : kb;
      (void)jcq;
      (void)kcq;
      const double wt = cw[q] + ((fv[q][0] + fv[q][1]) + fv[q][2]);  // face_at's order (0 where no face)
      v[q] += cp.omega * cd[q] * (cb[q] - wt);
    }
  }
  // per fine row of the block: its weights on coarse rows jb / jb + 1 (kb / kb + 1)
  double wy[2][2], wz[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const int j = 2 * jb + a, k = 2 * kb + a;
    rj[a] = j < x.fn[1];
    rk[a] = k < x.f_ke;
    wy[a][0] = wy[a][1] = wz[a][0] = wz[a][1] = 0.0;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      if (rj[a]) {
        const int ci = kld(x.pi[1], 2 * j + e);
        const double w = kld(x.pw[1], 2 * j + e);
        wy[a][0] += ci == jb ? w : 0.0;
        wy[a][1] += ci == jb + 1 ? w : 0.0;
      }
      if (rk[a]) {
        const int ci = kld(x.pi[2], 2 * k + e);
        const double w = kld(x.pw[2], 2 * k + e);
        wz[a][0] += ci == kb ? w : 0.0;
        wz[a][1] += ci == kb + 1 ? w : 0.0;
      }
    }
  }
  // x-interpolated coarse values: even fine node (coarse c), odd (c, c + 1)
  double e0[4], e1[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const double vr = shl1(v[q]);
    e0[q] = v[q];
    e1[q] = tail ? vr : wl * v[q] + wr * vr;
  }
  if (!has0) return;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int a = r & 1, b = r >> 1;
    if (!(rj[a] && rk[b])) continue;
    const double w00 = wz[b][0] * wy[a][0], w01 = wz[b][0] * wy[a][1];
    const double w10 = wz[b][1] * wy[a][0], w11 = wz[b][1] * wy[a][1];
    const double a0 = (w00 * e0[0] + w01 * e0[1]) + (w10 * e0[2] + w11 * e0[3]);
    const double a1 = (w00 * e1[0] + w01 * e1[1]) + (w10 * e1[2] + w11 * e1[3]);
    if (has1) {
      d2a8 out = {xo[r].x + a0, xo[r].y + a1};
      if (mask != nullptr) {
        const d2a8 m = ld_pair(mask + f[r]);
        if (m.x == 0.0) out.x = 0.0;
        if (m.y == 0.0) out.y = 0.0;
      }
      *reinterpret_cast<d2a8*>(xf + f[r]) = out;
    } else {
      const bool off = mask != nullptr && mask[f[r]] == 0.0;
      xf[f[r]] = off ? 0.0 : xo[r].x + a0;
    }
  }
}

template <int MODE, bool FACES>
__global__ __launch_bounds__(kBlock) void k_mg_jacobi(int64_t n, const PcgState* __restrict__ st,
                                                      const double* __restrict__ b, const double* __restrict__ w,
                                                      FaceAdd fa, const double* __restrict__ dinv, double omega,
                                                      double* __restrict__ x) {
  if (st != nullptr && st->done) return;
  const FaceRsrc fr = FACES ? face_rsrc(fa) : FaceRsrc{};
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < n; t += (int64_t)gridDim.x * kBlock) {
    if (MODE == 0) {
      x[t] = omega * dinv[t] * b[t];
    } else {
      double wt = w[t];
      if (FACES) wt += face_terms_nb(fa, fr, t);
      x[t] += omega * dinv[t] * (b[t] - wt);
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_mg_inject(MgXfer x, const double* __restrict__ Tf,
                                                      double* __restrict__ Tc, int nxb, int k0) {
  const int row = (int)blockIdx.x / nxb;
  const int i = ((int)blockIdx.x - row * nxb) * kBlock + (int)threadIdx.x;
  const int j = row % x.cn[1], k = k0 + row / x.cn[1];
  if (i >= x.cn[0]) return;
  // the fine node that coincides with coarse node (i, j, k): restriction entry 1 (weight 1)
  const int64_t f = x.ri[0][3 * i + 1] + (int64_t)x.fn[0] * (x.ri[1][3 * j + 1] + (int64_t)x.fn[1] * x.ri[2][3 * k + 1]);
  Tc[(int64_t)i + (int64_t)x.cn[0] * (j + (int64_t)x.cn[1] * k)] = Tf[f];
}

// the residual of a level in place of its J x, on the owned nodes of a
// partitioned level (pointers offset to the first owned node): w <- b - (w +
// facet terms); 0 where mask == 0 (Dirichlet-constrained rows).  The
// distributed V-cycle exchanges it and restricts it (tv_mgdist.cpp).
template <bool FACES>
__global__ __launch_bounds__(kBlock) void k_mg_resid(int64_t n, const PcgState* __restrict__ st,
                                                     const double* __restrict__ b, double* __restrict__ w, FaceAdd fa,
                                                     const double* __restrict__ mask) {
  if (st != nullptr && st->done) return;
  const FaceRsrc fr = FACES ? face_rsrc(fa) : FaceRsrc{};
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < n; t += (int64_t)gridDim.x * kBlock) {
    double wt = w[t];
    if (FACES) wt += face_terms_nb(fa, fr, t);
    const double d = b[t] - wt;
    w[t] = (mask != nullptr && mask[t] == 0.0) ? 0.0 : d;
  }
}

// restriction mask of a partitioned level: 1 on the owned nodes [own0, own1),
// 0 on the ghost planes (the ranks' partial restrictions then add up exactly)
// and on Dirichlet-constrained rows (dinv == 0, when dinv is given)
__global__ __launch_bounds__(kBlock) void k_mg_ownmask(int64_t n, int64_t own0, int64_t own1,
                                                       const double* __restrict__ dinv, double* __restrict__ mask) {
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < n; t += (int64_t)gridDim.x * kBlock)
    mask[t] = (t >= own0 && t < own1 && (dinv == nullptr || dinv[t] != 0.0)) ? 1.0 : 0.0;
}

// ---- DG1 level 0 <-> CG1 level 1 ------------------------------------------------------
// DG dof addressing of local cell layer k (DgGrid: a slab's owned layers
// first, [l][owned cell]; its ghost layers after them, [l][cell of the layer])
struct DgL {
  int64_t base, stride;
};
__device__ __forceinline__ DgL dg_lay(const DgGrid& g, int k) {
  const int64_t pc = (int64_t)g.c0 * g.c1;
  if (k < g.k_begin) return {g.gofs[0], pc};
  if (k >= g.k_end) return {g.gofs[1], pc};
  return {(int64_t)(k - g.k_begin) * pc, g.own};
}

// vertex (i, j, K) of local vertex plane K in [v0, v1): the sum of the
// cell-local copies (a, b, c) of the cells (i - a, j - b, K - c) whose layer
// lies in [ck0, ck1) (a slab: its owned layers; the ranks' partial sums on the
// shared vertex planes add up in the all-reduce of the replicated level), into
// the CG vector at global vertex plane K + kg0; with xc the CG level's
// pre-smoothing x = omega D^-1 b (one partition only: a partial sum is not b)
__global__ __launch_bounds__(kBlock) void k_mg_dg_restrict(DgGrid g, const PcgState* __restrict__ st,
                                                           const double* __restrict__ bf,
                                                           const double* __restrict__ wf,
                                                           const double* __restrict__ mask, double* __restrict__ bc,
                                                           const double* __restrict__ dinv_c, double omega_c,
                                                           double* __restrict__ xc, int v0, int v1, int ck0, int ck1,
                                                           int kg0) {
  if (st != nullptr && st->done) return;
  const int c0 = g.c0, c1 = g.c1, n0 = c0 + 1, n1 = c1 + 1;
  const int64_t nv = (int64_t)n0 * n1 * (v1 - v0);
  // (the mask test a compile-time choice: a load under a run-time test, even a
  // uniform one, ended in a wait for every load before it)
  auto run = [&](auto masked) {
    constexpr bool MASKED = decltype(masked)::value;
    for (int64_t v = blockIdx.x * (int64_t)kBlock + threadIdx.x; v < nv; v += (int64_t)gridDim.x * kBlock) {
      const int i = (int)(v % n0), j = (int)((v / n0) % n1), K = v0 + (int)(v / ((int64_t)n0 * n1));
      // the 8 cells' copies loaded together (clamped addresses, no branch around
      // a load), then summed in the same order over the cells that exist: with
      // a branch per copy each load waited for the one before (vmcnt counts in
      // order).  Adding +0.0 for a missing copy is exact (acc never is -0.0)
      const int64_t o = i + (int64_t)n0 * (j + (int64_t)n1 * (K + kg0));
      double bv[8], wv[8], mv[8];
      bool in[8];
#pragma unroll
      for (int l = 0; l < 8; ++l) {
        const int ci = i - (l & 1), cj = j - ((l >> 1) & 1), ck = K - (l >> 2);
        in[l] = !(ci < 0 || ci >= c0 || cj < 0 || cj >= c1 || ck < ck0 || ck >= ck1);
        const DgL a = dg_lay(g, min(max(ck, ck0), ck1 - 1));
        const int64_t f =
            a.base + (int64_t)l * a.stride + min(max(ci, 0), c0 - 1) + (int64_t)c0 * min(max(cj, 0), c1 - 1);
        bv[l] = bf[f];
        wv[l] = wf[f];
        mv[l] = MASKED ? mask[f] : 1.0;
      }
      double acc = 0.0;
#pragma unroll
      for (int l = 0; l < 8; ++l) acc += (in[l] && mv[l] != 0.0) ? bv[l] - wv[l] : 0.0;
      bc[o] = acc;
      if (xc != nullptr) xc[o] = omega_c * dinv_c[o] * acc;
    }
  };
  if (mask != nullptr) run(std::true_type{});
  else run(std::false_type{});
}

// every cell-local copy of the cells of local layers [ck0, ck1) takes its
// vertex value: x_dg(l, cell) += x_cg(vertex), the CG vector at global planes
// (a slab: its ghost layers too -- the replicated level holds every vertex)
__global__ __launch_bounds__(kBlock) void k_mg_dg_prolong(DgGrid g, const PcgState* __restrict__ st,
                                                          double* __restrict__ xf, const double* __restrict__ xc,
                                                          const double* __restrict__ mask, int ck0, int ck1, int kg0) {
  if (st != nullptr && st->done) return;
  const int c0 = g.c0, c1 = g.c1, n0 = c0 + 1, n1 = c1 + 1;
  const int64_t pc = (int64_t)c0 * c1, ncell = pc * (ck1 - ck0);
  auto run = [&](auto masked) {
    constexpr bool MASKED = decltype(masked)::value;
    for (int64_t cell = blockIdx.x * (int64_t)kBlock + threadIdx.x; cell < ncell; cell += (int64_t)gridDim.x * kBlock) {
      const int i = (int)(cell % c0), j = (int)((cell / c0) % c1), k = ck0 + (int)(cell / pc);
      const DgL a = dg_lay(g, k);
      // every load before the first store (a store to xf, then the next copy's
      // load from xf: the compiler cannot prove them apart, so each load waited
      // for the store and the load before it)
      double xv[8], cv[8], mv[8];
#pragma unroll
      for (int l = 0; l < 8; ++l) {
        const int64_t v = (i + (l & 1)) + (int64_t)n0 * ((j + ((l >> 1) & 1)) + (int64_t)n1 * (k + kg0 + (l >> 2)));
        const int64_t f = a.base + (int64_t)l * a.stride + i + (int64_t)c0 * j;
        xv[l] = xf[f];
        cv[l] = xc[v];
        mv[l] = MASKED ? mask[f] : 1.0;
      }
#pragma unroll
      for (int l = 0; l < 8; ++l) {
        const int64_t f = a.base + (int64_t)l * a.stride + i + (int64_t)c0 * j;
        xf[f] = (MASKED && mv[l] == 0.0) ? 0.0 : xv[l] + cv[l];
      }
    }
  };
  if (mask != nullptr) run(std::true_type{});
  else run(std::false_type{});
}

// T of the CG level: the mean of the cell-local copies at each vertex of local
// vertex planes [v0, v1) (over every local layer: a slab's ghost layers hold
// the neighbours' T), at global vertex plane K + kg0
__global__ __launch_bounds__(kBlock) void k_mg_dg_T(DgGrid g, const double* __restrict__ Tdg, double* __restrict__ Tcg,
                                                    int v0, int v1, int kg0) {
  const int c0 = g.c0, c1 = g.c1, c2 = g.c2, n0 = c0 + 1, n1 = c1 + 1;
  const int64_t nv = (int64_t)n0 * n1 * (v1 - v0);
  for (int64_t v = blockIdx.x * (int64_t)kBlock + threadIdx.x; v < nv; v += (int64_t)gridDim.x * kBlock) {
    const int i = (int)(v % n0), j = (int)((v / n0) % n1), K = v0 + (int)(v / ((int64_t)n0 * n1));
    double s = 0.0;
    int cnt = 0;
#pragma unroll
    for (int l = 0; l < 8; ++l) {
      const int ci = i - (l & 1), cj = j - ((l >> 1) & 1), ck = K - (l >> 2);
      if (ci < 0 || ci >= c0 || cj < 0 || cj >= c1 || ck < 0 || ck >= c2) continue;
      const DgL a = dg_lay(g, ck);
      s += Tdg[a.base + (int64_t)l * a.stride + ci + (int64_t)c0 * cj];
      ++cnt;
    }
    Tcg[i + (int64_t)n0 * (j + (int64_t)n1 * (K + kg0))] = s / cnt;
  }
}

__global__ __launch_bounds__(kBlock) void k_mg_pow(int64_t n, const double* __restrict__ dinv, double* __restrict__ y,
                                                   double* __restrict__ partials) {
  __shared__ double red[kBlock / kWave];
  double acc = 0.0;
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < n; t += (int64_t)gridDim.x * kBlock) {
    const double v = dinv ? dinv[t] * y[t] : y[t];  // null: the norm only
    y[t] = v;
    acc += v * v;
  }
  acc = wave_sum64(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) partials[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(kBlock) void k_mg_scale(int64_t n, const double* __restrict__ y, double a,
                                                     double* __restrict__ x) {
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < n; t += (int64_t)gridDim.x * kBlock) x[t] = a * y[t];
}

int blocks_for(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>((n + kBlock - 1) / kBlock, 8192)); }
// restriction: one coarse node per thread (27-point gathers: the coarse
// levels' few hundred blocks must not serialise rounds -- 4 nodes per thread
// measured 24 us at 143k coarse nodes)
int xfer_blocks(int64_t n) { return (int)std::max<int64_t>(1, (n + kBlock - 1) / kBlock); }

// ---- fused residual restriction (RRArgs, tv_internal.h) ----------------------
// A workgroup of kRRWaves waves = kRRWaves consecutive coarse rows Jc0 .. of the
// row axis, one 62-node coarse x segment and a chunk of coarse planes of the
// march axis.  Lane l holds coarse x node I = 62 seg - 1 + l and its fine pair
// (2I, 2I + 1) (the fine x cell count is even); the window 2I - 2 .. 2I + 2
// comes from lanes l - 1 / l + 1 by DPP (lanes 0 and 63 are halo lanes).  Per
// fine plane of the march window:
//   1. the workgroup's fine rows (2 kRRWaves + 3 on a coarsened row axis) are
//      loaded ONCE, spread over the waves (x and b as 16-byte pairs), the facet
//      terms subtracted from b on the face nodes, and each row x-reduced to
//        p = Rx Mx x,  q = Rx Kx x,  s = Rx (b - F x)
//      into a double-buffered LDS slab (one barrier per plane);
//   2. each wave folds its coarse row's five fine rows from the slab:
//        U = RrMr (p + da q) + da RrKr p,  V = RrMr p,  S = Rr s
//      and accumulates b_c(Q) = sum over the window of Rq S - RqMq U - da RqKq V
//      (two accumulators: an even plane 2k completes coarse k - 2, opens k).
// The loads of planes P + 1 .. P + kRRPF are in flight while plane P is reduced
// and folded (a ring of kRRPF + 1 register sets; one workgroup per CU, so the
// ring's registers cost no occupancy).
constexpr int kRRSeg = kWave - 2;
constexpr int kRRWaves = 8;
constexpr int kRRRows = 2 * kRRWaves + 3;          // fine rows per plane (coarsened row axis)
constexpr int kRRPer = (kRRRows + kRRWaves - 1) / kRRWaves;  // rows loaded per wave
constexpr int kRRQMax = 64;  // coarse march planes per chunk (LDS weight stage)
constexpr int kRRPF = 1;     // fine planes of loads in flight ahead of the one reduced (2, 3: slower, profiles/r06_rrestrict_loads_ab.txt)

// buffer resource of a level vector (32-bit byte offsets: a per-lane x offset in
// a VGPR plus a wave-uniform row / plane offset in an SGPR)
using rr_buf = __amdgpu_buffer_rsrc_t;
__device__ __forceinline__ rr_buf rr_rsrc(const void* p, uint32_t bytes) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  void* q = (void*)(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(q, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
__device__ __forceinline__ d2a8 rr_ld2(rr_buf r, uint32_t voff, uint32_t soff) {
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  const u4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, (int)soff, 0);
  return __builtin_bit_cast(d2a8, v);
}
__device__ __forceinline__ double rr_ld1(rr_buf r, uint32_t voff) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, (int)voff, 0, 0));
}

// one fine plane's loads; every load is issued unconditionally (lanes / waves
// without the data carry an out-of-range offset): a load under a branch made
// the wave wait for all its loads there (vmcnt counts in order), i.e. for the
// prefetch of the next planes too
struct RRSet {
  d2a8 xv[kRRPer], bv[kRRPer];
  double fx[kRRPer];  // the x-face facet term of each row at this lane's node (x-face lanes only)
  d2a8 fr;            // the row-axis face term of this wave's face row (waves holding one)
};

template <int RA>
__global__ __launch_bounds__(kRRWaves * kWave) void k_mg_rrestrict(RRArgs a, const PcgState* __restrict__ st,
                                                                   const double* __restrict__ b,
                                                                   const double* __restrict__ x, FaceAdd fa,
                                                                   double* __restrict__ bc,
                                                                   const double* __restrict__ dinv_c, double omega_c,
                                                                   double* __restrict__ xc) {
  if (st != nullptr && st->done) return;
  __shared__ double sq[kRRQMax][15];        // the chunk's march-axis windows
  __shared__ double sr[kRRWaves][15];       // each wave's row-axis window
  __shared__ double red[2][3][kRRRows][kWave];  // x-reduced rows (p, q, s), two planes
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  constexpr int ra = RA, qa = 3 - RA;
  const int ncr = a.cn[ra], ncq = a.cn[qa];
  const int nrb = (ncr + kRRWaves - 1) / kRRWaves;
  // order: x segment fastest, then row block, then chunk; contiguous per XCD
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int seg = bid % a.nseg;
  const int t = bid / a.nseg;
  const int rb = t % nrb, chunk = t / nrb;
  const int Jc0 = rb * kRRWaves;
  const int Jc = Jc0 + wave;
  const bool row_ok = Jc < ncr;
  const int Jcc = row_ok ? Jc : ncr - 1;
  const int Q0 = chunk * a.qchunk, Q1 = min(Q0 + a.qchunk, ncq);
  const int nf0 = a.fn[0], ncx = a.cn[0];
  const int nfr = a.fn[ra], nfq = a.fn[qa];
  const int I = seg * kRRSeg - 1 + lane;
  const bool Iok = I >= 0 && I < ncx;
  const int e0 = 2 * I;
  {
    const int tid = threadIdx.x;
    for (int e = tid; e < 15 * (Q1 - Q0); e += kRRWaves * kWave) sq[e / 15][e % 15] = a.ax[qa].w[15 * Q0 + e];
    if (lane < 15) sr[wave][lane] = row_ok ? a.ax[ra].w[15 * Jcc + lane] : 0.0;
  }
  // the workgroup's fine rows: fr_first .. fr_first + nrows - 1 (clamped to the axis)
  const int Jlast = min(Jc0 + kRRWaves, ncr) - 1;
  const int fr_first = kld(a.ax[ra].f0, Jc0);
  const int nrows = kld(a.ax[ra].f0, Jlast) + 5 - fr_first;  // <= kRRRows (rr_setup)
  const int my0 = kld(a.ax[ra].f0, Jcc) - fr_first;           // this wave's first row in the slab
  const int sR = (ra == 1) ? nf0 : nf0 * a.fn[1];
  const int sQ = (ra == 1) ? nf0 * a.fn[1] : nf0;
  // the rows this wave loads: slab rows wave, wave + kRRWaves, ...
  int frow[kRRPer];
  uint32_t rowoff[kRRPer];
  bool rload[kRRPer];
#pragma unroll
  for (int u = 0; u < kRRPer; ++u) {
    const int sl = wave + u * kRRWaves;
    rload[u] = sl < nrows;
    frow[u] = min(max(fr_first + sl, 0), nfr - 1);  // clamped (weight 0 outside the axis)
    rowoff[u] = (uint32_t)(sR * frow[u]) * 8u;
  }
  const uint32_t nbytes = (uint32_t)a.fn[0] * (uint32_t)a.fn[1] * (uint32_t)a.fn[2] * 8u;
  const rr_buf rx = rr_rsrc(x, nbytes), rbv = rr_rsrc(b, nbytes);
  // the lane's fine pair (e0, e0 + 1) straight from the row; the last lane's
  // e0 + 1 is the next row's first node (weight 0), the lanes outside the axis
  // carry an out-of-range offset (the range check returns 0)
  const uint32_t voff = Iok ? (uint32_t)e0 * 8u : 0x40000000u;
  // facet terms: the x faces at the lanes holding fine x node 0 / nf0 - 1 (in
  // the waves that have one: loaded with the plane), the row-axis faces on the
  // axis' first / last row and the march-axis faces on the first / last fine
  // plane (wave-uniform branches, rare)
  const bool xl0 = fa.ff[0] != nullptr && e0 == 0, xl1 = fa.ff[1] != nullptr && e0 == nf0 - 1;
  const int n1 = a.fn[1];
  // the two x-face arrays through one resource: they lie in one allocation
  // (CgGrid::ffbuf), face 1 at a uniform element distance from face 0
  const double* fxb = fa.ff[0] ? fa.ff[0] : fa.ff[1];
  const int64_t dx1 = (fa.ff[0] && fa.ff[1]) ? (int64_t)(fa.ff[1] - fa.ff[0]) : 0;
  const rr_buf rfx = rr_rsrc(fxb, fxb ? (uint32_t)((dx1 + (int64_t)n1 * a.fn[2]) * 8) : 0u);
  const uint32_t fxo = xl1 ? (uint32_t)dx1 : 0u;
  const uint32_t nfa = nbytes / (uint32_t)nfr, nfb = nbytes / (uint32_t)nfq;  // face array bytes
  const rr_buf frl = rr_rsrc(fa.ff[2 * ra], fa.ff[2 * ra] ? nfa : 0u);
  const rr_buf frh = rr_rsrc(fa.ff[2 * ra + 1], fa.ff[2 * ra + 1] ? nfa : 0u);
  const rr_buf fql = rr_rsrc(fa.ff[2 * qa], fa.ff[2 * qa] ? nfb : 0u);
  const rr_buf fqh = rr_rsrc(fa.ff[2 * qa + 1], fa.ff[2 * qa + 1] ? nfb : 0u);
  const bool hrl = fa.ff[2 * ra] != nullptr, hrh = fa.ff[2 * ra + 1] != nullptr;
  const bool hql = fa.ff[2 * qa] != nullptr, hqh = fa.ff[2 * qa + 1] != nullptr;
  // this wave's face row among its loaded rows (wave-uniform; at most one: the
  // face rows are the first and the last of the axis)
  int uf = -1;
  bool uf_lo = false;
#pragma unroll
  for (int u = 0; u < kRRPer; ++u) {
    const int fr = fr_first + wave + u * kRRWaves;
    if (rload[u] && ((hrl && fr == 0) || (hrh && fr == nfr - 1))) {
      uf = u;
      uf_lo = hrl && fr == 0;
    }
  }
  const rr_buf frs = uf_lo ? frl : frh;
  const int f0q = kld(a.ax[qa].f0, Q0);
  const int np = 2 * (Q1 - Q0) + 3;  // fine planes f0q .. f0q + np - 1
  auto fetch = [&](int P, RRSet& S) {
    const int fq = min(max(f0q + P, 0), nfq - 1);
    const uint32_t po = (uint32_t)(sQ * fq) * 8u;
#pragma unroll
    for (int u = 0; u < kRRPer; ++u) {
      S.xv[u] = rr_ld2(rx, rload[u] ? voff : 0x40000000u, rowoff[u] + po);
      S.bv[u] = rr_ld2(rbv, rload[u] ? voff : 0x40000000u, rowoff[u] + po);
    }
#pragma unroll
    for (int u = 0; u < kRRPer; ++u) {
      // storage (j, k) of (row frow[u], plane fq): the x-face index j + n1 k
      const int j = (ra == 1) ? frow[u] : fq, k = (ra == 1) ? fq : frow[u];
      S.fx[u] = rr_ld1(rfx, ((xl0 || xl1) && rload[u]) ? (fxo + (uint32_t)(j + n1 * k)) * 8u : 0x40000000u);
    }
    // the face row's pairs (face index i + n0 * plane)
    S.fr = rr_ld2(frs, uf >= 0 ? voff : 0x40000000u, (uint32_t)(nf0 * fq) * 8u);
  };
  // the lane's x weights in registers (read for every loaded row)
  double wx[15];
#pragma unroll
  for (int m = 0; m < 15; ++m) wx[m] = (Iok ? a.ax[0].w[15 * (Iok ? I : 0) + m] : 0.0);
  // the loaded rows of plane P: facet terms, x-reduction into slab buffer P & 1
  auto reduce = [&](int P, const RRSet& S) {
    const int fqr = f0q + P;
    const bool qlo = hql && fqr == 0, qhi = hqh && fqr == nfq - 1;  // wave-uniform
    d2a8 sv[kRRPer];
#pragma unroll
    for (int u = 0; u < kRRPer; ++u) {
      sv[u] = S.bv[u];
      sv[u].x -= S.fx[u];
      if (u == uf) {  // a row-axis face row (wave-uniform)
        sv[u].x -= S.fr.x;
        sv[u].y -= S.fr.y;
      }
      if (qlo || qhi) {  // a march-axis face plane (face index i + n0 * row)
        const d2a8 f = rr_ld2(qlo ? fql : fqh, voff, (uint32_t)(nf0 * frow[u]) * 8u);
        sv[u].x -= f.x;
        sv[u].y -= f.y;
      }
    }
    const int buf = P & 1;
#pragma unroll
    for (int u = 0; u < kRRPer; ++u) {
      const d2a8 xv = S.xv[u];
      // x window (2I - 2, 2I - 1, 2I, 2I + 1, 2I + 2)
      const double x0 = shr1(xv.x), x1 = shr1(xv.y), x4 = shl1(xv.x);
      const double s0 = shr1(sv[u].x), s1 = shr1(sv[u].y), s4 = shl1(sv[u].x);
      const double p = ((wx[0] * x0 + wx[1] * x1) + wx[2] * xv.x) + (wx[3] * xv.y + wx[4] * x4);
      const double q = ((wx[5] * x0 + wx[6] * x1) + wx[7] * xv.x) + (wx[8] * xv.y + wx[9] * x4);
      const double s = ((wx[10] * s0 + wx[11] * s1) + wx[12] * sv[u].x) + (wx[13] * sv[u].y + wx[14] * s4);
      const int sl = wave + u * kRRWaves;
      if (sl < kRRRows) {  // (compile-time true for all but the last u)
        red[buf][0][sl][lane] = p;
        red[buf][1][sl][lane] = q;
        red[buf][2][sl][lane] = s;
      }
    }
  };
  // this wave's coarse row from the slab: (U, V, S)
  auto fold = [&](int P, double& U, double& V, double& Sv) {
    const int buf = P & 1;
    double um = 0.0, uk = 0.0, vv = 0.0, ss = 0.0;
#pragma unroll
    for (int m = 0; m < 5; ++m) {
      const int sl = min(my0 + m, kRRRows - 1);
      const double p = red[buf][0][sl][lane], q = red[buf][1][sl][lane], s = red[buf][2][sl][lane];
      um += sr[wave][m] * (p + a.da * q);
      uk += sr[wave][5 + m] * p;
      vv += sr[wave][m] * p;
      ss += sr[wave][10 + m] * s;
    }
    U = um + a.da * uk;
    V = vv;
    Sv = ss;
  };
  // window-position contribution of a fine plane to coarse plane Q (weights of Q's window slot m)
  auto contrib = [&](int Q, int m, double U, double V, double Sv) {
    const double* w = sq[Q - Q0];
    return w[10 + m] * Sv - (w[m] * U + a.da * (w[5 + m] * V));
  };
  const bool out_lane = row_ok && Iok && lane >= 1 && lane <= kRRSeg;
  const int nQ = Q1 - Q0;
  // fine plane P feeds coarse planes Q0 + k with 2k <= P <= 2k + 4.  X = the
  // older, Y = the newer live coarse plane; an even plane 2k completes coarse
  // k - 2 (written out) and opens coarse k.
  double X = 0.0, Y = 0.0;
  // D^-1 of the coarse node an even plane completes, loaded at the start of
  // that plane's step (ahead of its prefetch, so waiting for it does not wait
  // for the prefetch: a load at the store made every even plane wait for all)
  const uint32_t ncb = (uint32_t)ncx * (uint32_t)a.cn[1] * (uint32_t)a.cn[2] * 8u;
  const rr_buf rdc = rr_rsrc(dinv_c, xc != nullptr ? ncb : 0u);
  auto coarse_off = [&](int Q) -> uint32_t {
    const int J1 = (ra == 1) ? Jc : Q, K2 = (ra == 1) ? Q : Jc;
    return ((uint32_t)I + (uint32_t)ncx * ((uint32_t)J1 + (uint32_t)a.cn[1] * (uint32_t)K2)) * 8u;
  };
  RRSet S[kRRPF + 1];
#pragma unroll
  for (int s = 0; s < kRRPF; ++s) fetch(min(s, np - 1), S[s]);
  __syncthreads();  // the weight stages
  // slot s of the ring holds plane P0 + s when step s of the unrolled group
  // starts; it fetches plane P0 + s + kRRPF into the slot consumed one step ago
  // (planes past the chunk are clamped reloads, never reduced)
#pragma unroll 1
  for (int P0 = 0; P0 < np; P0 += kRRPF + 1) {
#pragma unroll
    for (int s = 0; s <= kRRPF; ++s) {
      const int P = P0 + s;
      const bool completes = P < np && (P & 1) == 0 && (P >> 1) - 2 >= 0 && out_lane;
      const double dcv = rr_ld1(rdc, completes ? coarse_off(Q0 + (P >> 1) - 2) : 0x40000000u);
      __builtin_amdgcn_sched_barrier(0);  // issued ahead of the prefetch (vmcnt counts in order)
      fetch(min(P + kRRPF, np - 1), S[(s + kRRPF) % (kRRPF + 1)]);
      if (P < np) {  // workgroup-uniform
        reduce(P, S[s]);
        __syncthreads();
        double U, V, Sv;
        fold(P, U, V, Sv);
        const int k = P >> 1;
        if ((P & 1) == 0) {
          if (k - 2 >= 0 && k - 2 < nQ) X += contrib(Q0 + k - 2, 4, U, V, Sv);
          if (k - 1 >= 0 && k - 1 < nQ) Y += contrib(Q0 + k - 1, 2, U, V, Sv);
          const double Z = (k < nQ) ? contrib(Q0 + k, 0, U, V, Sv) : 0.0;
          if (completes) {  // coarse Q0 + k - 2 complete
            const int64_t o = coarse_off(Q0 + k - 2) / 8u;
            bc[o] = X;
            if (xc != nullptr) xc[o] = omega_c * dcv * X;  // the coarse pre-smoothing step from 0
          }
          X = Y;
          Y = Z;
        } else {
          if (k - 1 >= 0 && k - 1 < nQ) X += contrib(Q0 + k - 1, 3, U, V, Sv);
          if (k < nQ) Y += contrib(Q0 + k, 1, U, V, Sv);
        }
      }
    }
  }
}

}  // namespace



void launch_mg_restrict(const MgXfer& x, const PcgState* st, const double* bf, const double* wf, const FaceAdd* fa,
                        const double* mask, double* bc, const double* dinv_c, double omega_c, double* xc,
                        hipStream_t s) {
  // fa (on): wf lacks the face-workgroup facet terms, added here (only where
  // mg_restrict_folds_faces(x): the caller checks, see mg_level in tv_api.cpp)
  const bool faces = fa != nullptr && fa->on;
  const int64_t n = (int64_t)x.cn[0] * x.cn[1] * (x.c_ke - x.c_kb);
  if (n <= 0) return;
  if (mg_restrict_folds_faces(x)) {  // by rows, 16-byte fine pairs
    const int nseg = (x.cn[0] + kPairSeg - 1) / kPairSeg;
    const dim3 g((unsigned)((int64_t)x.cn[1] * (x.c_ke - x.c_kb) * nseg));
    const FaceAdd f = faces ? *fa : FaceAdd{};
#define TV_RP(M, F) \
  hipLaunchKernelGGL((k_mg_restrict_pairs<M, F>), g, dim3(kWave), 0, s, x, st, bf, wf, mask, bc, dinv_c, omega_c, xc, \
                     nseg, f)
    if (mask != nullptr) {
      if (faces) TV_RP(true, true);
      else TV_RP(true, false);
    } else {
      if (faces) TV_RP(false, true);
      else TV_RP(false, false);
    }
#undef TV_RP
    return;
  }
  if (mask != nullptr)
    hipLaunchKernelGGL(k_mg_restrict<true>, dim3(xfer_blocks(n)), dim3(kBlock), 0, s, x, st, bf, wf, mask, bc, dinv_c,
                       omega_c, xc);
  else
    hipLaunchKernelGGL(k_mg_restrict<false>, dim3(xfer_blocks(n)), dim3(kBlock), 0, s, x, st, bf, wf, mask, bc,
                       dinv_c, omega_c, xc);
}

bool mg_restrict_folds_faces(const MgXfer& x) { return x.coarse[0] && x.fn[0] >= 3; }

void launch_mg_rrestrict(const RRArgs& a, const PcgState* st, const double* b, const double* x, const FaceAdd& fa,
                         double* bc, const double* dinv_c, double omega_c, double* xc, hipStream_t s) {
  const int ncr = a.cn[a.raxis], ncq = a.cn[3 - a.raxis];
  const int nrb = (ncr + kRRWaves - 1) / kRRWaves;
  if (a.qchunk > kRRQMax) return;  // (rr_setup keeps it below)
  const int nch = (ncq + a.qchunk - 1) / a.qchunk;
  const dim3 g((unsigned)((int64_t)a.nseg * nrb * nch)), bl(kRRWaves * kWave);
  if (a.raxis == 1) hipLaunchKernelGGL(k_mg_rrestrict<1>, g, bl, 0, s, a, st, b, x, fa, bc, dinv_c, omega_c, xc);
  else hipLaunchKernelGGL(k_mg_rrestrict<2>, g, bl, 0, s, a, st, b, x, fa, bc, dinv_c, omega_c, xc);
}

bool mg_prolong_blocks(const MgXfer& x) {
  return x.aligned && x.coarse[0] && x.coarse[1] && x.coarse[2] && x.fn[0] >= 3 && x.f_kb == 0;
}

bool mg_prolong_smooths(const MgXfer& x) { return mg_prolong_blocks(x); }

void launch_mg_prolong(const MgXfer& x, const PcgState* st, double* xf, const double* xc, const double* mask,
                       hipStream_t s, const CoarsePost* cp) {
  const int64_t n = (int64_t)x.fn[0] * x.fn[1] * (x.f_ke - x.f_kb);
  if (n <= 0) return;
  if (cp != nullptr && !mg_prolong_smooths(x)) {
    // not reached (mg_prolong_from asks mg_prolong_smooths first); kept correct
    // anyway: the coarse post-smoothing step in place, then the plain prolongation
    const int64_t nc = (int64_t)x.cn[0] * x.cn[1] * x.cn[2];
    launch_mg_jacobi(nc, st, cp->b, cp->w, &cp->fa, cp->dinv, cp->omega, const_cast<double*>(xc), 1, s);
    cp = nullptr;
  }
  if (mg_prolong_blocks(x)) {  // 2 x 2 blocks of fine rows, 16-byte fine pairs
    const int nseg = ((x.fn[0] + 1) / 2 + kPairSeg - 1) / kPairSeg;
    const int nbj = (x.fn[1] + 1) / 2, nbk = (x.f_ke + 1) / 2;
    if (cp != nullptr)
      hipLaunchKernelGGL(k_mg_prolong_blk<true>, dim3((unsigned)((int64_t)nbj * nbk * nseg)), dim3(kWave), 0, s, x, st,
                         xf, xc, mask, nseg, nbj, *cp);
    else
      hipLaunchKernelGGL(k_mg_prolong_blk<false>, dim3((unsigned)((int64_t)nbj * nbk * nseg)), dim3(kWave), 0, s, x, st,
                         xf, xc, mask, nseg, nbj, CoarsePost{});
    return;
  }
  if (x.coarse[0] && x.fn[0] >= 3) {  // by rows, 16-byte fine pairs
    const int nseg = ((x.fn[0] + 1) / 2 + kPairSeg - 1) / kPairSeg;
    const int64_t rows = (int64_t)x.fn[1] * (x.f_ke - x.f_kb);
    hipLaunchKernelGGL(k_mg_prolong_pairs, dim3((unsigned)(rows * nseg)), dim3(kWave), 0, s, x, st, xf, xc, mask, nseg);
    return;
  }
  hipLaunchKernelGGL(k_mg_prolong, dim3((unsigned)((n + kPU * kBlock - 1) / (kPU * kBlock))), dim3(kBlock), 0, s, x, st, xf, xc, mask);
}

void launch_mg_jacobi(int64_t n, const PcgState* st, const double* b, const double* w, const FaceAdd* fa,
                      const double* dinv, double omega, double* x, int mode, hipStream_t s) {
  if (n <= 0) return;
  const FaceAdd f = (fa && fa->on) ? *fa : FaceAdd{};
  const dim3 g(blocks_for(n)), bl(kBlock);
  if (mode == 0) hipLaunchKernelGGL((k_mg_jacobi<0, false>), g, bl, 0, s, n, st, b, w, f, dinv, omega, x);
  else if (f.on) hipLaunchKernelGGL((k_mg_jacobi<1, true>), g, bl, 0, s, n, st, b, w, f, dinv, omega, x);
  else hipLaunchKernelGGL((k_mg_jacobi<1, false>), g, bl, 0, s, n, st, b, w, f, dinv, omega, x);
}

void launch_mg_inject(const MgXfer& x, const double* Tf, double* Tc, hipStream_t s) {
  launch_mg_inject_range(x, Tf, Tc, 0, x.cn[2], s);
}

void launch_mg_inject_range(const MgXfer& x, const double* Tf, double* Tc, int k0, int k1, hipStream_t s) {
  const int nxb = (x.cn[0] + kBlock - 1) / kBlock;
  const int64_t rows = (int64_t)x.cn[1] * (k1 - k0);
  if (rows > 0) hipLaunchKernelGGL(k_mg_inject, dim3((unsigned)(rows * nxb)), dim3(kBlock), 0, s, x, Tf, Tc, nxb, k0);
}

void launch_mg_resid(int64_t n, const PcgState* st, const double* b, double* w, const FaceAdd* fa, const double* mask,
                     hipStream_t s) {
  if (n <= 0) return;
  const FaceAdd f = (fa && fa->on) ? *fa : FaceAdd{};
  if (f.on) hipLaunchKernelGGL((k_mg_resid<true>), dim3(blocks_for(n)), dim3(kBlock), 0, s, n, st, b, w, f, mask);
  else hipLaunchKernelGGL((k_mg_resid<false>), dim3(blocks_for(n)), dim3(kBlock), 0, s, n, st, b, w, f, mask);
}

void launch_mg_ownmask(int64_t n, int64_t own0, int64_t own1, const double* dinv, double* mask, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_mg_ownmask, dim3(blocks_for(n)), dim3(kBlock), 0, s, n, own0, own1, dinv, mask);
}

// the vertex planes of the CG level a DG slab writes (DgRange): one
// partition -- every plane; a slab -- the planes of its owned layers (their
// restriction, the shared planes as partial sums) or its owned vertex planes
// (vertex plane K belongs to the owner of layer K, the last one to the last slab)
void launch_mg_dg_restrict(const DgGrid& g, const PcgState* st, const double* bf, const double* wf, const double* mask,
                           double* bc, const double* dinv_c, double omega_c, double* xc, int kg0, hipStream_t s) {
  const int64_t nv = (int64_t)(g.c0 + 1) * (g.c1 + 1) * (g.k_end - g.k_begin + 1);
  hipLaunchKernelGGL(k_mg_dg_restrict, dim3(blocks_for(nv)), dim3(kBlock), 0, s, g, st, bf, wf, mask, bc, dinv_c,
                     omega_c, xc, g.k_begin, g.k_end + 1, g.k_begin, g.k_end, kg0);
}

void launch_mg_dg_prolong(const DgGrid& g, const PcgState* st, double* xf, const double* xc, const double* mask,
                          int kg0, hipStream_t s) {
  const int64_t nc = (int64_t)g.c0 * g.c1 * g.c2;
  hipLaunchKernelGGL(k_mg_dg_prolong, dim3(blocks_for(nc)), dim3(kBlock), 0, s, g, st, xf, xc, mask, 0, g.c2, kg0);
}

void launch_mg_dg_T(const DgGrid& g, const double* Tdg, double* Tcg, int kg0, hipStream_t s) {
  const int v1 = g.k_end + (g.gofs[1] < 0 ? 1 : 0);  // the top vertex plane: the last slab's
  const int64_t nv = (int64_t)(g.c0 + 1) * (g.c1 + 1) * (v1 - g.k_begin);
  hipLaunchKernelGGL(k_mg_dg_T, dim3(blocks_for(nv)), dim3(kBlock), 0, s, g, Tdg, Tcg, g.k_begin, v1, kg0);
}

int launch_mg_pow(int64_t n, const double* dinv, double* y, double* partials, hipStream_t s) {
  const int nb = (int)std::max<int64_t>(1, std::min<int64_t>((n + kBlock - 1) / kBlock, 1024));
  hipLaunchKernelGGL(k_mg_pow, dim3(nb), dim3(kBlock), 0, s, n, dinv, y, partials);
  return nb;
}

void launch_mg_scale(int64_t n, const double* y, double a, double* x, hipStream_t s) {
  hipLaunchKernelGGL(k_mg_scale, dim3(blocks_for(n)), dim3(kBlock), 0, s, n, y, a, x);
}

}  // namespace tv
