// CG1 (Q1 quadrilateral / hexahedral) operators on UNSTRUCTURED meshes, gfx950:
// the path for meshes that are not tensor-product grids (gmsh .msh input,
// distorted cells).
//
// Replaces, for such meshes, the FFCx cell kernel of F dx and its Jacobian
// (ThermoViscoProblem.py:295-300, ufl.derivative at :331), the exterior-facet
// kernels of the Robin terms (:302-304) and the assembled PETSc matrix that
// dolfinx's NonlinearProblem hands to KSP (:331-343) [3P].
//
// Design (measured).  A matrix-free isoparametric J x --
// 27 Gauss points per hexahedron, the Jacobian, its inverse and the physical
// gradients at each -- costs ~16 kflop per cell: fp64-FLOP bound, 2.6 ms per
// J x at 8M cells (2 % of the HBM roofline of its 72 B per cell).  The cell
// part of J(T) is M + dt alpha K, independent of T, so it is assembled ONCE at
// context creation into SELL-64 (sliced ELLPACK: 64-row slices = one
// wavefront, column-major inside a slice, so the value / column loads of a
// wave are 512 B / 256 B coalesced) and J x streams 12 B per stored entry
// (~27 per row) at HBM speed.  The T-dependent Robin terms are evaluated on
// the fly, row by row, from per-facet quadrature weights w_q |J_s| stored at
// setup (boundary rows only).  Every row is owned by one lane: no atomics, no
// colouring, the summation order is fixed (bitwise reproducible).
//  * J x  (japply / the fused PCG matvec): V = M + dt alpha K;
//  * F(T) (residual): M (T - T_prev) + (dt alpha K) T - dt f int phi + Robin, with
//    M and dt alpha K kept apart so T - T_prev is formed before the product
//    (no cancellation at T ~ T_prev);
//  * diag J: diag V + the Robin diagonal.
// Assembly: one thread per row gathers the rows of the element matrices of the
// cells around its vertex (3-point Gauss per direction and the isoparametric
// Jacobian, the oracle's rule, oracle/tv_oracle.py HeatForm) in cell order.
#include <algorithm>
#include <cstdio>
#include <thread>
#include <vector>

#include "tv_device.h"

namespace tv {

struct UmDevice {
  std::vector<void*> bufs;            // freed by um_free
  std::vector<unsigned char> bmask;   // host: vertices on the boundary
  int64_t nnz = 0;                    // stored entries (incl. SELL padding)
  int64_t nb = 0;                     // boundary vertices
};

namespace {

enum { UM_RES = 0, UM_JAC = 1, UM_DIAG = 2, UM_FUSED = 3 };
constexpr int kUmBlocksMax = 2048;  // grid cap of the row kernels (partial records of the fused launch)

__device__ constexpr double kUX[3] = {0.11270166537925831148, 0.5, 0.88729833462074168852};
__device__ constexpr double kUW[3] = {5.0 / 18.0, 8.0 / 18.0, 5.0 / 18.0};

__device__ __forceinline__ double um_g(const UmGrid& g, double T) {
  const double T2 = T * T;
  return g.a_rad * (T2 * T2 - g.T_amb4) + g.a_conv * (T - g.T_amb);
}
__device__ __forceinline__ double um_dg(const UmGrid& g, double T) { return g.a_rad * 4.0 * (T * T * T) + g.a_conv; }

// Q1 basis and reference gradients at xi (tensor order l = a + 2b + 4c)
template <int D>
__device__ __forceinline__ void q1(const double (&xi)[3], double (&phi)[1 << D], double (&dphi)[1 << D][D]) {
#pragma unroll
  for (int l = 0; l < (1 << D); ++l) {
    double f[3], df[3];
#pragma unroll
    for (int a = 0; a < D; ++a) {
      const int b = (l >> a) & 1;
      f[a] = b ? xi[a] : 1.0 - xi[a];
      df[a] = b ? 1.0 : -1.0;
    }
    double p = 1.0;
#pragma unroll
    for (int a = 0; a < D; ++a) p *= f[a];
    phi[l] = p;
#pragma unroll
    for (int a = 0; a < D; ++a) {
      double q = df[a];
#pragma unroll
      for (int e = 0; e < D; ++e)
        if (e != a) q *= f[e];
      dphi[l][a] = q;
    }
  }
}

// inverse and determinant of a D x D matrix
template <int D>
__device__ __forceinline__ double inv_det(const double (&J)[D][D], double (&Ji)[D][D]) {
  if constexpr (D == 2) {
    const double det = J[0][0] * J[1][1] - J[0][1] * J[1][0];
    const double id = 1.0 / det;
    Ji[0][0] = J[1][1] * id;
    Ji[0][1] = -J[0][1] * id;
    Ji[1][0] = -J[1][0] * id;
    Ji[1][1] = J[0][0] * id;
    return det;
  } else {
    double c[3][3];
    c[0][0] = J[1][1] * J[2][2] - J[1][2] * J[2][1];
    c[0][1] = J[0][2] * J[2][1] - J[0][1] * J[2][2];
    c[0][2] = J[0][1] * J[1][2] - J[0][2] * J[1][1];
    c[1][0] = J[1][2] * J[2][0] - J[1][0] * J[2][2];
    c[1][1] = J[0][0] * J[2][2] - J[0][2] * J[2][0];
    c[1][2] = J[0][2] * J[1][0] - J[0][0] * J[1][2];
    c[2][0] = J[1][0] * J[2][1] - J[1][1] * J[2][0];
    c[2][1] = J[0][1] * J[2][0] - J[0][0] * J[2][1];
    c[2][2] = J[0][0] * J[1][1] - J[0][1] * J[1][0];
    const double det = J[0][0] * c[0][0] + J[0][1] * c[1][0] + J[0][2] * c[2][0];
    const double id = 1.0 / det;
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int b = 0; b < 3; ++b) Ji[a][b] = c[a][b] * id;
    return det;
  }
}


// ---- setup kernels -----------------------------------------------------------------
// row l of the element matrices of a cell: Ml[j] = int phi_l phi_j,
// Kl[j] = int grad phi_l . grad phi_j
template <int D>
__device__ __forceinline__ void elem_row(const double (&X)[1 << D][D], int l, double (&Ml)[1 << D],
                                         double (&Kl)[1 << D]) {
  constexpr int NL = 1 << D;
  constexpr int NQ = (D == 2) ? 9 : 27;
#pragma unroll
  for (int j = 0; j < NL; ++j) Ml[j] = Kl[j] = 0.0;
#pragma unroll 1
  for (int q = 0; q < NQ; ++q) {
    const int qi[3] = {q % 3, (q / 3) % 3, q / 9};
    double xi[3] = {0.0, 0.0, 0.0}, w = 1.0;
#pragma unroll
    for (int a = 0; a < D; ++a) {
      xi[a] = kUX[qi[a]];
      w *= kUW[qi[a]];
    }
    double phi[NL], dphi[NL][D];
    q1<D>(xi, phi, dphi);
    double J[D][D];
#pragma unroll
    for (int a = 0; a < D; ++a)
#pragma unroll
      for (int b = 0; b < D; ++b) {
        double s = 0.0;
#pragma unroll
        for (int m = 0; m < NL; ++m) s += X[m][a] * dphi[m][b];
        J[a][b] = s;
      }
    double Ji[D][D];
    const double wd = w * fabs(inv_det<D>(J, Ji));
    double gp[NL][D];  // grad phi = J^-T dphi
#pragma unroll
    for (int m = 0; m < NL; ++m)
#pragma unroll
      for (int a = 0; a < D; ++a) {
        double s = 0.0;
#pragma unroll
        for (int b = 0; b < D; ++b) s += Ji[b][a] * dphi[m][b];
        gp[m][a] = s;
      }
    double phil = 0.0, gl[D];
#pragma unroll
    for (int a = 0; a < D; ++a) gl[a] = 0.0;
#pragma unroll
    for (int m = 0; m < NL; ++m)
      if (m == l) {
        phil = phi[m];
#pragma unroll
        for (int a = 0; a < D; ++a) gl[a] = gp[m][a];
      }
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      double gg = 0.0;
#pragma unroll
      for (int a = 0; a < D; ++a) gg += gl[a] * gp[j][a];
      Ml[j] += wd * (phil * phi[j]);
      Kl[j] += wd * gg;
    }
  }
}

// one thread per row: sums the element rows of the cells around the vertex
// (incidences in cell order) into the row's SELL entries, then V = M + K,
// diag V and int phi_r
template <int D>
__global__ __launch_bounds__(kBlock) void k_um_assemble(int64_t nv, int64_t nc, const int* __restrict__ cell,
                                                        const double* __restrict__ X0, const double* __restrict__ X1,
                                                        const double* __restrict__ X2,
                                                        const int64_t* __restrict__ inc_off,
                                                        const int64_t* __restrict__ inc,
                                                        const int64_t* __restrict__ soff, const int* __restrict__ cols,
                                                        const int* __restrict__ rnnz, double dt_alpha,
                                                        double* __restrict__ V, double* __restrict__ M,
                                                        double* __restrict__ K, double* __restrict__ bvec,
                                                        double* __restrict__ vdiag) {
  constexpr int NL = 1 << D;
  const int64_t r = blockIdx.x * (int64_t)kBlock + threadIdx.x;
  if (r >= nv) return;
  const int64_t base = soff[r >> 6] + (r & 63);
  const int nz = rnnz[r];
  const double* Xa[3] = {X0, X1, X2};
  for (int64_t t = inc_off[r]; t < inc_off[r + 1]; ++t) {
    const int64_t e = inc[t] >> 3;
    const int l = (int)(inc[t] & 7);
    int nd[NL];
    double X[NL][D];
#pragma unroll
    for (int m = 0; m < NL; ++m) {
      nd[m] = cell[(int64_t)m * nc + e];
#pragma unroll
      for (int a = 0; a < D; ++a) X[m][a] = Xa[a][nd[m]];
    }
    double Ml[NL], Kl[NL];
    elem_row<D>(X, l, Ml, Kl);
#pragma unroll
    for (int j = 0; j < NL; ++j) {
      int lo = 0, hi = nz;  // columns of the row are sorted
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (cols[base + 64 * (int64_t)mid] < nd[j]) lo = mid + 1;
        else hi = mid;
      }
      const int64_t idx = base + 64 * (int64_t)lo;
      M[idx] += Ml[j];
      K[idx] += dt_alpha * Kl[j];
    }
  }
  double b = 0.0;
  for (int k = 0; k < nz; ++k) {
    const int64_t idx = base + 64 * (int64_t)k;
    const double v = M[idx] + K[idx];
    V[idx] = v;
    b += M[idx];
    if (cols[idx] == (int)r) vdiag[r] = v;
  }
  bvec[r] = b;
}

// one thread per boundary facet: its vertex ids in facet-local tensor order
// and w_q |J_s|(q) = w_q |det J| |J^-T e_n| at its 3^(d-1) points (the
// oracle's facet measure)
template <int D>
__global__ __launch_bounds__(kBlock) void k_um_facet_setup(int64_t nf, int64_t nc, const int* __restrict__ fcell,
                                                           const signed char* __restrict__ flf,
                                                           const int* __restrict__ cell, const double* __restrict__ X0,
                                                           const double* __restrict__ X1,
                                                           const double* __restrict__ X2, int* __restrict__ fv,
                                                           double* __restrict__ fw) {
  constexpr int NL = 1 << D;
  constexpr int NQ = (D == 2) ? 3 : 9;
  const int64_t f = blockIdx.x * (int64_t)kBlock + threadIdx.x;
  if (f >= nf) return;
  const int64_t e = fcell[f];
  const int lf = flf[f];
  const int ax = lf >> 1, side = lf & 1;
  const double* Xa[3] = {X0, X1, X2};
  double X[NL][D];
  int m = 0;
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    const int v = cell[(int64_t)l * nc + e];
#pragma unroll
    for (int a = 0; a < D; ++a) X[l][a] = Xa[a][v];
    if (((l >> ax) & 1) == side) fv[(int64_t)(m++) * nf + f] = v;
  }
#pragma unroll 1
  for (int q = 0; q < NQ; ++q) {
    double xi[3] = {0.0, 0.0, 0.0}, w = 1.0;
    int t = 0;
#pragma unroll
    for (int a = 0; a < D; ++a) {
      if (a == ax) {
        xi[a] = (double)side;
        continue;
      }
      const int qi = (t == 0) ? (q % 3) : (q / 3);
      xi[a] = kUX[qi];
      w *= kUW[qi];
      ++t;
    }
    double phi[NL], dphi[NL][D];
    q1<D>(xi, phi, dphi);
    double J[D][D];
#pragma unroll
    for (int a = 0; a < D; ++a)
#pragma unroll
      for (int b = 0; b < D; ++b) {
        double s = 0.0;
#pragma unroll
        for (int l = 0; l < NL; ++l) s += X[l][a] * dphi[l][b];
        J[a][b] = s;
      }
    double Ji[D][D];
    const double det = fabs(inv_det<D>(J, Ji));
    double gn = 0.0;  // |row ax of J^-1| = |grad xi_ax|
#pragma unroll
    for (int b = 0; b < D; ++b) gn += Ji[ax][b] * Ji[ax][b];
    fw[(int64_t)q * nf + f] = w * det * sqrt(gn);
  }
}

// ---- the row kernels ---------------------------------------------------------------
// facet-local Q1 basis at facet point q: tangential axes in increasing order,
// point index q = i0 + 3 i1 (the product order of q1<D> on the cell)
__device__ __forceinline__ double fphi(int m, int q, int D) {
  const double x0 = kUX[q % 3];
  const double f0 = (m & 1) ? x0 : 1.0 - x0;
  if (D == 2) return f0;
  const double x1 = kUX[q / 3];
  return f0 * ((m >> 1) ? x1 : 1.0 - x1);
}

// Robin terms of row r (ThermoViscoProblem.py:302-304 and their derivative)
template <int D, int MODE, class XGet>
__device__ __forceinline__ double robin_row(const UmGrid& g, int64_t r, const double* __restrict__ T, XGet xget) {
  constexpr int NF = 1 << (D - 1);
  constexpr int NQ = (D == 2) ? 3 : 9;
  double acc = 0.0;
  const int t1 = g.boff[r + 1];
  for (int t = g.boff[r]; t < t1; ++t) {
    const int code = g.binc[t];
    const int64_t f = code >> 2;
    const int m = code & 3;
    double Tn[NF], xn[NF];
#pragma unroll
    for (int n = 0; n < NF; ++n) {
      const int v = g.fv[(int64_t)n * g.nf + f];
      Tn[n] = T[v];
      xn[n] = (MODE == UM_JAC || MODE == UM_FUSED) ? xget(v) : 0.0;
    }
    double y = 0.0;
#pragma unroll 1
    for (int q = 0; q < NQ; ++q) {
      double Tq = 0.0, xq = 0.0, pm = 0.0;
#pragma unroll
      for (int n = 0; n < NF; ++n) {
        const double ph = fphi(n, q, D);
        Tq += ph * Tn[n];
        xq += ph * xn[n];
        if (n == m) pm = ph;
      }
      double v;
      if (MODE == UM_RES) v = um_g(g, Tq) * pm;
      else if (MODE == UM_DIAG) v = um_dg(g, Tq) * pm * pm;
      else v = um_dg(g, Tq) * xq * pm;
      y += g.fw[(int64_t)q * g.nf + f] * v;
    }
    acc += g.dt * y;
  }
  return acc;
}

// One lane per row, one wave per 64-row slice, each wave a contiguous range of
// slices (XCD-remapped blocks: a contiguous row range per XCD, so the x
// gathers of neighbouring rows share one L2).
//   UM_JAC:   out = V u + Robin'(T) u
//   UM_FUSED: the same with u = p (formed by k_um_pvec), out = w, p.w records
//             + the reduction tail (PETSc's dpi and alpha)
//   UM_RES:   out = M (u - up) + K u - dt f b + Robin(u)      (u = T, up = T_prev)
//   UM_DIAG:  out = diag V + Robin diagonal (inverted if `invert`)
template <int D, int MODE>
__global__ __launch_bounds__(kBlock) void k_um_rows(UmGrid g, const double* __restrict__ T,
                                                    const double* __restrict__ u, const double* __restrict__ up,
                                                    double* __restrict__ out, const PcgState* __restrict__ st,
                                                    double* __restrict__ partials, RedTail rt, int invert) {
  if (MODE == UM_FUSED && st->done) return;
  auto xget = [&](int64_t c) -> double { return u[c]; };
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int WPB = kBlock / 64;
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t nw = (int64_t)gridDim.x * WPB;
  const int64_t gw = (int64_t)blk * WPB + wave;
  const int64_t chunk = (g.nslice + nw - 1) / nw;
  const int64_t s0 = gw * chunk, s1 = std::min<int64_t>(s0 + chunk, g.nslice);
  double pw = 0.0;
  for (int64_t s = s0; s < s1; ++s) {
    const int64_t r = s * 64 + lane;
    const int64_t so = g.soff[s];
    const int wdt = (int)((g.soff[s + 1] - so) >> 6);
    const int* __restrict__ cs = g.cols + so + lane;  // entry k of this row: cs[64 k]
    double acc = 0.0, acc2 = 0.0;
    if (MODE == UM_RES) {
      const double* __restrict__ ms = g.M + so + lane;
      const double* __restrict__ ks = g.K + so + lane;
      for (int k = 0; k < wdt; ++k) {
        const int c = __builtin_nontemporal_load(&cs[64 * k]);
        const double xc = u[c];
        acc += __builtin_nontemporal_load(&ms[64 * k]) * (xc - up[c]);
        acc2 += __builtin_nontemporal_load(&ks[64 * k]) * xc;
      }
    } else if (MODE != UM_DIAG) {
      const double* __restrict__ vs = g.V + so + lane;
      // U entries in flight per lane and round, the last round masked (27
      // entries per interior hexahedral row = 3 full rounds of 9).  The matrix
      // stream is read once per product: non-temporal loads keep it from
      // evicting the gathered vector from L2 / the Infinity Cache (measured at
      // 8.2M rows: 598 vs 717 us per J x, 4.6 vs 3.8 TB/s)
      constexpr int U = 9;
      for (int k = 0; k < wdt; k += U) {
        int c[U];
        double a[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
          const bool ok = k + j < wdt;
          const int o = 64 * (ok ? k + j : 0);
          c[j] = __builtin_nontemporal_load(&cs[o]);
          a[j] = __builtin_nontemporal_load(&vs[o]);
          if (!ok) a[j] = 0.0;
        }
#pragma unroll
        for (int j = 0; j < U; ++j) acc += a[j] * u[c[j]];
      }
    }
    if (r < g.nrow) {
      double val;
      if (MODE == UM_DIAG) val = g.vdiag[r];
      else if (MODE == UM_RES) val = (acc + acc2) - g.dt_f * g.bvec[r];
      else val = acc;
      // Robin terms: the residual's in a pass over the boundary rows of their
      // own (k_um_robin_res: no divergent facet quadrature in this kernel's
      // waves); structured topology runs J x on the half stencil instead
      // (k_um_march14, the Robin Jacobian folded in)
      if (MODE != UM_RES)
        val += robin_row<D, MODE>(g, r, T, xget);
      if (MODE == UM_DIAG && invert) val = 1.0 / val;
      if (MODE == UM_FUSED) pw += u[r] * val;
      out[r] = val;
    }
  }
  if (MODE == UM_FUSED) {
    __shared__ double red[WPB];
    const double sw = wave_sum64(pw);
    if (lane == 0) red[wave] = sw;
    __syncthreads();
    if (threadIdx.x == 0) store_partial(&partials[blockIdx.x], (red[0] + red[1]) + (red[2] + red[3]));
    fused_reduce_tail<1>(rt, gridDim.x);
  }
}

// PETSc KSPCG "p <- z + (beta / betaold) p" (p = z at iteration 0) into the
// buffer of this iteration's parity (the convention of k_pcg_update); carries
// the start stamp of the iteration's matvec
__global__ __launch_bounds__(kBlock) void k_um_pvec(int64_t n, const PcgState* __restrict__ st,
                                                    const double* __restrict__ z, double* pA, double* pB,
                                                    int it_host, RedTail rt) {
  stamp_start(rt);
  if (st->done) return;
  const bool first = it_host == 0;
  const double b = first ? 0.0 : st->beta / st->betaold;
  double* p = (it_host & 1) ? pB : pA;
  const double* po = (it_host & 1) ? pA : pB;
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < n; t += (int64_t)gridDim.x * kBlock)
    p[t] = first ? z[t] : z[t] + b * po[t];
}

// the residual's Robin terms (ThermoViscoProblem.py:302-304) on the boundary rows,
// added to the cell part k_um_rows<UM_RES> wrote: F[r] = (cell part) + Robin,
// the same association as a single pass
template <int D>
__global__ __launch_bounds__(kBlock) void k_um_robin_res(UmGrid g, const double* __restrict__ u, double* __restrict__ F) {
  auto xget = [&](int64_t c) -> double { return u[c]; };
  for (int64_t b = blockIdx.x * (int64_t)kBlock + threadIdx.x; b < g.nbr; b += (int64_t)gridDim.x * kBlock) {
    const int64_t r = g.brow[b];
    F[r] += robin_row<D, UM_RES>(g, r, u, xget);
  }
}

// the owned values the neighbours hold as ghosts, gathered into the send buffer
__global__ __launch_bounds__(kBlock) void k_um_pack(const int64_t* __restrict__ idx, int64_t n,
                                                    const double* __restrict__ v, double* __restrict__ out) {
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < n; t += (int64_t)gridDim.x * kBlock) out[t] = v[idx[t]];
}

int row_blocks(const UmGrid& g) {
  return (int)std::max<int64_t>(1, std::min<int64_t>((g.nslice + 3) / 4, kUmBlocksMax));
}

// Structured topology: the half-stencil J x with one wave per column of rows --
// an x segment of 64 vertices at row j -- marching the planes k (in kch chunks
// of the plane axis).  Row r's lower slots a plane back are the upper slots of
// rows this wave read one plane step earlier (L1 / L2 hits; in row order they
// come back ~160K rows later and miss, 72 B per row), and the neighbouring
// columns j +- 1 run on the same XCD (consecutive waves).
struct March14 {
  int64_t n0, n1, n2;
  int nseg, kch, kper;
  int64_t ncol;
};
March14 march14(const UmGrid& g) {
  March14 m;
  m.n0 = g.s1;
  m.n1 = g.s2 / g.s1;
  m.n2 = g.nv / g.s2;
  m.nseg = (int)((m.n0 + 63) / 64);
  m.ncol = (int64_t)m.nseg * m.n1;
  // enough waves for the chip (>= ~4K), at most 4 chunks of the plane axis
  m.kch = (int)std::max<int64_t>(1, std::min<int64_t>({4, m.n2, (4096 + m.ncol - 1) / m.ncol}));
  m.kper = (int)((m.n2 + m.kch - 1) / m.kch);
  return m;
}
int march_blocks(const UmGrid& g) {
  if (g.J14 == nullptr) return 1;
  const March14 m = march14(g);
  return (int)std::max<int64_t>(1, std::min<int64_t>((m.ncol * m.kch + 3) / 4, kUmBlocksMax));
}

template <int MODE>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4))) void k_um_march14(UmGrid g, March14 m, const double* __restrict__ u,
                                                       double* __restrict__ out, const PcgState* __restrict__ st,
                                                       double* __restrict__ partials, RedTail rt) {
  if (MODE == UM_FUSED && st->done) return;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int WPB = kBlock / 64;
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t nw = (int64_t)gridDim.x * WPB;
  double pw = 0.0;
  for (int64_t gw = (int64_t)blk * WPB + wave; gw < m.ncol * m.kch; gw += nw) {
    const int64_t seg = gw % m.nseg, t = gw / m.nseg;  // segment fastest, then row j, then chunk
    const int64_t j = t % m.n1, ch = t / m.n1;
    const int64_t i = seg * 64 + lane;
    if (i >= m.n0) continue;
    const int64_t k1 = std::min<int64_t>(m.n2, (ch + 1) * m.kper);
    // 32-bit unsigned element indices (14 nv < 2^31 and 8 x that < 2^32: checked
    // at setup): uniform base + 32-bit offset loads, no 64-bit address VGPRs
    const double* __restrict__ J = g.J14;
    const unsigned nv = (unsigned)g.nv, s1 = (unsigned)g.s1, s2 = (unsigned)g.s2;
#pragma unroll 1
    for (int64_t k = ch * m.kper; k < k1; ++k) {
      const unsigned r = (unsigned)(i + m.n0 * j + g.s2 * k);
      double acc = 0.0;
#pragma unroll
      for (int q14 = 0; q14 < 14; ++q14) {
        const int q = 13 + q14;
        const unsigned o = (unsigned)(q % 3 - 1) + s1 * (unsigned)((q / 3) % 3 - 1) + s2 * (unsigned)(q / 9 - 1);
        const bool hi = r + o < nv, lo = r >= o;  // (o >= 0 for the upper slots)
        const unsigned cu = hi ? r + o : r, cl = lo ? r - o : r;
        const unsigned ku = (unsigned)q14 * nv;
        acc += J[ku + r] * u[cu];
        if (q14 > 0) acc += (lo ? J[ku + cl] : 0.0) * u[cl];
      }
      out[r] = acc;
      if (MODE == UM_FUSED) pw += u[r] * acc;
    }
  }
  if (MODE == UM_FUSED) {
    __shared__ double red[WPB];
    const double sw = wave_sum64(pw);
    if (lane == 0) red[wave] = sw;
    __syncthreads();
    if (threadIdx.x == 0) store_partial(&partials[blockIdx.x], (red[0] + red[1]) + (red[2] + red[3]));
    fused_reduce_tail<1>(rt, gridDim.x);
  }
}

// The residual's cell part on the half stencils of M and dt alpha K (structured
// topology), marched like k_um_march14: F = M (T - T_prev) + K T - dt f b (the
// same grouping as k_um_rows<UM_RES>, M and K apart so T - T_prev is formed
// first); the Robin terms follow in k_um_robin_res
__global__ __launch_bounds__(kBlock) void k_um_res14(UmGrid g, March14 m, const double* __restrict__ u,
                                                       const double* __restrict__ up, double* __restrict__ out) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int WPB = kBlock / 64;
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t nw = (int64_t)gridDim.x * WPB;
  const double* __restrict__ Mh = g.M14;
  const double* __restrict__ Kh = g.K14;
  const unsigned nv = (unsigned)g.nv, s1 = (unsigned)g.s1, s2 = (unsigned)g.s2;
  for (int64_t gw = (int64_t)blk * WPB + wave; gw < m.ncol * m.kch; gw += nw) {
    const int64_t seg = gw % m.nseg, t = gw / m.nseg;
    const int64_t j = t % m.n1, ch = t / m.n1;
    const int64_t i = seg * 64 + lane;
    if (i >= m.n0) continue;
    const int64_t k1 = std::min<int64_t>(m.n2, (ch + 1) * m.kper);
#pragma unroll 1
    for (int64_t k = ch * m.kper; k < k1; ++k) {
      const unsigned r = (unsigned)(i + m.n0 * j + g.s2 * k);
      double acc = 0.0, acc2 = 0.0;
#pragma unroll 7
      for (int q14 = 0; q14 < 14; ++q14) {
        const int q = 13 + q14;
        const unsigned o = (unsigned)(q % 3 - 1) + s1 * (unsigned)((q / 3) % 3 - 1) + s2 * (unsigned)(q / 9 - 1);
        const bool hi = r + o < nv, lo = r >= o;
        const unsigned cu = hi ? r + o : r, cl = lo ? r - o : r;
        const unsigned ku = (unsigned)q14 * nv;
        const double xu = u[cu];
        acc += Mh[ku + r] * (xu - up[cu]);
        acc2 += Kh[ku + r] * xu;
        if (q14 > 0) {
          const double xl = u[cl];
          acc += (lo ? Mh[ku + cl] : 0.0) * (xl - up[cl]);
          acc2 += (lo ? Kh[ku + cl] : 0.0) * xl;
        }
      }
      out[r] = (acc + acc2) - g.dt_f * g.bvec[r];
    }
  }
}

template <int MODE>
void launch_rows(const UmGrid& g, const double* T, const double* u, const double* up, double* out,
                 const PcgState* st, double* partials, const RedTail& rt, int invert, hipStream_t s) {
  const dim3 grid(row_blocks(g)), block(kBlock);
  if (g.dim == 2)
    hipLaunchKernelGGL((k_um_rows<2, MODE>), grid, block, 0, s, g, T, u, up, out, st, partials, rt, invert);
  else
    hipLaunchKernelGGL((k_um_rows<3, MODE>), grid, block, 0, s, g, T, u, up, out, st, partials, rt, invert);
}

}  // namespace

// A structured grid's half-stencil operator, one row per thread (the small
// coarse grids of the geometric hierarchy: every row in flight at once);
// POST: the damped Jacobi step y = x + omega dinv (b - A x)
template <bool POST>
__global__ __launch_bounds__(kBlock) void k_sg_rows(UmGrid g, const PcgState* __restrict__ st,
                                                   const double* __restrict__ x, const double* __restrict__ b,
                                                   const double* __restrict__ dinv, double omega,
                                                   double* __restrict__ y) {
  if (st != nullptr && st->done) return;
  const double* __restrict__ J = g.J14;
  const unsigned nv = (unsigned)g.nv, s1 = (unsigned)g.s1, s2 = (unsigned)g.s2;
  for (unsigned r = blockIdx.x * kBlock + threadIdx.x; r < nv; r += gridDim.x * kBlock) {
    double acc = 0.0;
#pragma unroll
    for (int k = 0; k < 14; ++k) {
      const int q = 13 + k;
      const unsigned o = (unsigned)(q % 3 - 1) + s1 * (unsigned)((q / 3) % 3 - 1) + s2 * (unsigned)(q / 9 - 1);
      const bool hi = r + o < nv, lo = r >= o;
      const unsigned cu = hi ? r + o : r, cl = lo ? r - o : r;
      const unsigned ku = (unsigned)k * nv;
      acc += J[ku + r] * x[cu];
      if (k > 0) acc += (lo ? J[ku + cl] : 0.0) * x[cl];
    }
    y[r] = POST ? x[r] + omega * dinv[r] * (b[r] - acc) : acc;
  }
}

// ---- index-space transfers of the geometric hierarchy (level 0) ----------------
// per axis: fine node i is kept (a coarse node) when even or the last one; a
// kept node's coarse index is i / 2, the odd last one's nc - 1; the others
// interpolate their two kept neighbours at 1/2 (tv_amg.cpp geometric_p)
struct GeoDims {
  int f[3], c[3];
};
__device__ __forceinline__ int geo_cidx(int i, int nf, int nc) { return (i == nf - 1 && (i & 1)) ? nc - 1 : i >> 1; }
__device__ __forceinline__ bool geo_kept(int i, int nf) { return !(i & 1) || i == nf - 1; }

// b_c[I] = sum over the (<= 3)^3 fine nodes that interpolate from I, one thread per coarse node
__global__ __launch_bounds__(kBlock) void k_geo_restrict0(GeoDims d, const PcgState* __restrict__ st,
                                                          const double* __restrict__ r,
                                                          const double* __restrict__ dinv_c, double omega_c,
                                                          double* __restrict__ b_c, double* __restrict__ x_c) {
  if (st != nullptr && st->done) return;
  const int64_t nc = (int64_t)d.c[0] * d.c[1] * d.c[2];
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < nc; t += (int64_t)gridDim.x * kBlock) {
    const int ci[3] = {(int)(t % d.c[0]), (int)((t / d.c[0]) % d.c[1]), (int)(t / ((int64_t)d.c[0] * d.c[1]))};
    int fi[3][3];
    double wi[3][3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const int nf = d.f[a];
      const int f = (ci[a] == d.c[a] - 1 && ((nf - 1) & 1)) ? nf - 1 : 2 * ci[a];
      fi[a][0] = f - 1; fi[a][1] = f; fi[a][2] = f + 1;
      wi[a][0] = (f - 1 >= 0 && !geo_kept(f - 1, nf)) ? 0.5 : 0.0;
      wi[a][1] = 1.0;
      wi[a][2] = (f + 1 < nf && !geo_kept(f + 1, nf)) ? 0.5 : 0.0;
      if (wi[a][0] == 0.0) fi[a][0] = f;
      if (wi[a][2] == 0.0) fi[a][2] = f;
    }
    double acc = 0.0;
#pragma unroll
    for (int kk = 0; kk < 3; ++kk)
#pragma unroll
      for (int jj = 0; jj < 3; ++jj) {
        double row = 0.0;
        const int64_t base = (int64_t)d.f[0] * (fi[1][jj] + (int64_t)d.f[1] * fi[2][kk]);
#pragma unroll
        for (int ii = 0; ii < 3; ++ii) row += wi[0][ii] * r[base + fi[0][ii]];
        acc += (wi[2][kk] * wi[1][jj]) * row;
      }
    b_c[t] = acc;
    if (x_c) x_c[t] = omega_c * dinv_c[t] * acc;
  }
}

// z = x0 + P x_c, one thread per fine node; (z.z, z.r) per workgroup and the tail
__global__ __launch_bounds__(kBlock) void k_geo_prolong0(GeoDims d, const PcgState* __restrict__ st,
                                                         const double* __restrict__ x_c,
                                                         const double* __restrict__ x0, const double* __restrict__ r,
                                                         double* __restrict__ z, double* __restrict__ partials,
                                                         RedTail rt) {
  if (st->done) return;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  constexpr int WPB = kBlock / 64;
  const int blk = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t nf = (int64_t)d.f[0] * d.f[1] * d.f[2];
  const int64_t per = ((nf + gridDim.x - 1) / gridDim.x + 63) / 64 * 64;  // a contiguous range per workgroup
  const int64_t t0 = (int64_t)blk * per, t1 = std::min<int64_t>(t0 + per, nf);
  double zz = 0.0, zr = 0.0;
  for (int64_t t = t0 + threadIdx.x; t < t1; t += kBlock) {
    const int fi[3] = {(int)(t % d.f[0]), (int)((t / d.f[0]) % d.f[1]), (int)(t / ((int64_t)d.f[0] * d.f[1]))};
    int c[3][2];
    double w[3][2];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const int i = fi[a], n = d.f[a], m = d.c[a];
      if (geo_kept(i, n)) {
        c[a][0] = c[a][1] = geo_cidx(i, n, m);
        w[a][0] = 1.0;
        w[a][1] = 0.0;
      } else {
        c[a][0] = geo_cidx(i - 1, n, m);
        c[a][1] = geo_cidx(i + 1, n, m);
        w[a][0] = w[a][1] = 0.5;
      }
    }
    double acc = 0.0;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int64_t base = (int64_t)d.c[0] * (c[1][jj] + (int64_t)d.c[1] * c[2][kk]);
        const double row = w[0][0] * x_c[base + c[0][0]] + w[0][1] * x_c[base + c[0][1]];
        acc += (w[2][kk] * w[1][jj]) * row;
      }
    const double zv = x0[t] + acc;
    z[t] = zv;
    zz += zv * zv;
    zr += zv * r[t];
  }
  __shared__ double red[2][WPB];
  const double s_zz = wave_sum64(zz), s_zr = wave_sum64(zr);
  if (lane == 0) {
    red[0][wave] = s_zz;
    red[1][wave] = s_zr;
  }
  __syncthreads();
  if (threadIdx.x < 2)
    store_partial(&partials[2 * (int64_t)blockIdx.x + threadIdx.x],
                  (red[threadIdx.x][0] + red[threadIdx.x][1]) + (red[threadIdx.x][2] + red[threadIdx.x][3]));
  fused_reduce_tail<2>(rt, gridDim.x);
}

GeoDims geo_dims(const int64_t (&fn)[3], const int64_t (&cn)[3]) {
  GeoDims d;
  for (int a = 0; a < 3; ++a) {
    d.f[a] = (int)fn[a];
    d.c[a] = (int)cn[a];
  }
  return d;
}

void launch_geo_restrict0(const int64_t (&fn)[3], const int64_t (&cn)[3], const PcgState* st, const double* r,
                          const double* dinv_c, double omega_c, double* b_c, double* x_c, hipStream_t s) {
  const int64_t nc = cn[0] * cn[1] * cn[2];
  const dim3 gr((unsigned)std::max<int64_t>(1, std::min<int64_t>((nc + kBlock - 1) / kBlock, 8192)));
  hipLaunchKernelGGL(k_geo_restrict0, gr, dim3(kBlock), 0, s, geo_dims(fn, cn), st, r, dinv_c, omega_c, b_c, x_c);
}

int launch_geo_prolong0(const int64_t (&fn)[3], const int64_t (&cn)[3], const PcgState* st, const double* x_c,
                        const double* x0, const double* r, double* z, double* partials, const RedTail* tail,
                        hipStream_t s) {
  const int64_t nf = fn[0] * fn[1] * fn[2];
  const int nb = (int)std::max<int64_t>(1, std::min<int64_t>((nf + kBlock - 1) / kBlock, kUmBlocksMax));
  const RedTail rt = tail ? *tail : RedTail{};
  hipLaunchKernelGGL(k_geo_prolong0, dim3(nb), dim3(kBlock), 0, s, geo_dims(fn, cn), st, x_c, x0, r, z, partials, rt);
  return nb;
}

void launch_sg_apply(const UmGrid& g, const PcgState* st, const double* x, const double* b, const double* dinv,
                     double omega, double* y, hipStream_t s) {
  // (the plane-marching kernel of the fine level on these grids: V-cycle 351-355
  // vs 320-324 us at distorted C4 -- 7 planes per wave, too few to pay)
  const dim3 gr((unsigned)std::max<int64_t>(1, std::min<int64_t>((g.nv + kBlock - 1) / kBlock, 8192)));
  if (b) hipLaunchKernelGGL(k_sg_rows<true>, gr, dim3(kBlock), 0, s, g, st, x, b, dinv, omega, y);
  else hipLaunchKernelGGL(k_sg_rows<false>, gr, dim3(kBlock), 0, s, g, st, x, nullptr, nullptr, 0.0, y);
}

int um_num_blocks(const UmGrid& g) { return std::max(row_blocks(g), march_blocks(g)); }
Sell um_operator(const UmGrid& g) {
  Sell m;
  m.nrow = g.nrow;
  m.ncol = g.nv;
  m.nslice = g.nslice;
  m.soff = g.soff;
  m.cols = g.cols;
  m.vals = g.V;
  return m;
}
void launch_um_pack(const int64_t* idx, int64_t n, const double* v, double* out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_um_pack, dim3((unsigned)std::min<int64_t>(1024, (n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                     idx, n, v, out);
}
int64_t um_nnz(const UmDevice* d) { return d ? d->nnz : 0; }
int64_t um_boundary_vertices(const UmDevice* d, std::vector<unsigned char>& mask) {
  mask = d->bmask;
  return d->nb;
}

void launch_um_residual(const UmGrid& g, const double* T, const double* Tp, double* F, hipStream_t s) {
  if (g.M14 != nullptr)
    hipLaunchKernelGGL(k_um_res14, dim3(march_blocks(g)), dim3(kBlock), 0, s, g, march14(g), T, Tp, F);
  else
    launch_rows<UM_RES>(g, T, T, Tp, F, nullptr, nullptr, RedTail{}, 0, s);
  if (g.nbr == 0) return;
  const dim3 gr((unsigned)std::max<int64_t>(1, std::min<int64_t>((g.nbr + kBlock - 1) / kBlock, 4096)));
  if (g.dim == 2) hipLaunchKernelGGL(k_um_robin_res<2>, gr, dim3(kBlock), 0, s, g, T, F);
  else hipLaunchKernelGGL(k_um_robin_res<3>, gr, dim3(kBlock), 0, s, g, T, F);
}

void launch_um_japply(const UmGrid& g, const double* T, const double* x, double* y, hipStream_t s) {
  if (g.J14 != nullptr) {
    hipLaunchKernelGGL(k_um_march14<UM_JAC>, dim3(march_blocks(g)), dim3(kBlock), 0, s, g, march14(g), x, y,
                       nullptr, nullptr, RedTail{});
    return;
  }
  launch_rows<UM_JAC>(g, T, x, nullptr, y, nullptr, nullptr, RedTail{}, 0, s);
}

void launch_um_diag(const UmGrid& g, const double* T, double* d, int invert, hipStream_t s) {
  launch_rows<UM_DIAG>(g, T, nullptr, nullptr, d, nullptr, nullptr, RedTail{}, invert, s);
}

int launch_um_japply_fused(const UmGrid& g, const double* T, const double* z, double* pA, double* pB, double* w,
                           const PcgState* st, double* partials, int it_host, const RedTail* tail, hipStream_t s) {
  const RedTail rt = tail ? *tail : RedTail{};
  const int vb = (int)std::max<int64_t>(1, std::min<int64_t>((g.nv + kBlock - 1) / kBlock, 2048));
  hipLaunchKernelGGL(k_um_pvec, dim3(vb), dim3(kBlock), 0, s, g.nv, st, z, pA, pB, it_host, rt);
  const double* p = (it_host & 1) ? pB : pA;
  if (g.J14 != nullptr) {
    const int nb = march_blocks(g);
    hipLaunchKernelGGL(k_um_march14<UM_FUSED>, dim3(nb), dim3(kBlock), 0, s, g, march14(g), p, w, st, partials, rt);
    return nb;
  }
  launch_rows<UM_FUSED>(g, T, p, nullptr, w, st, partials, rt, 0, s);
  return row_blocks(g);
}

// J14 = V14 + the Robin facet Jacobian dt int_f g'(T_h) phi_r phi_m ds of each
// boundary row r (the terms robin_row<UM_JAC> applies to x), one thread per
// boundary row: its 14 upper slots copied from V14, then per boundary incidence
// the 3^(d-1)-point facet quadrature accumulated into the upper slots of the
// facet's vertices (race-free: a row's slots belong to its thread; the lower
// couplings are the upper slots of the facet's other rows, which are boundary
// rows too)
__global__ __launch_bounds__(kBlock) void k_um_robin_fold(UmGrid g, const double* __restrict__ T) {
  constexpr int NF = 4, NQ = 9;
  for (int64_t b = blockIdx.x * (int64_t)kBlock + threadIdx.x; b < g.nbr; b += (int64_t)gridDim.x * kBlock) {
    const int64_t r = g.brow[b];
#pragma unroll
    for (int k = 0; k < 14; ++k) g.J14[(int64_t)k * g.nv + r] = g.V14[(int64_t)k * g.nv + r];
    const int t1 = g.boff[r + 1];
    for (int t = g.boff[r]; t < t1; ++t) {
      const int code = g.binc[t];
      const int64_t f = code >> 2;
      const int m = code & 3;
      double Tn[NF];
      int64_t vn[NF];
#pragma unroll
      for (int n = 0; n < NF; ++n) {
        vn[n] = g.fv[(int64_t)n * g.nf + f];
        Tn[n] = T[vn[n]];
      }
      double cn[NF] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll 1
      for (int q = 0; q < NQ; ++q) {
        double Tq = 0.0, pm = 0.0, ph[NF];
#pragma unroll
        for (int n = 0; n < NF; ++n) {
          ph[n] = fphi(n, q, 3);
          Tq += ph[n] * Tn[n];
          if (n == m) pm = ph[n];
        }
        const double wq = g.fw[(int64_t)q * g.nf + f] * um_dg(g, Tq) * pm;
#pragma unroll
        for (int n = 0; n < NF; ++n) cn[n] += wq * ph[n];
      }
#pragma unroll
      for (int n = 0; n < NF; ++n) {
        const int64_t off = vn[n] - r;
        const int64_t dk = (off + g.s2 / 2 + g.s2) / g.s2 - 1;
        const int64_t rem = off - dk * g.s2;
        const int64_t dj = (rem + g.s1 / 2 + g.s1) / g.s1 - 1;
        const int64_t di = rem - dj * g.s1;
        const int sl = (int)((di + 1) + 3 * (dj + 1) + 9 * (dk + 1));
        if (sl >= 13) g.J14[(int64_t)(sl - 13) * g.nv + r] += g.dt * cn[n];
      }
    }
  }
}

void launch_um_robin_fold(const UmGrid& g, const double* T, hipStream_t s) {
  if (g.J14 == nullptr || g.nbr == 0) return;
  const int nb = (int)std::max<int64_t>(1, std::min<int64_t>((g.nbr + kBlock - 1) / kBlock, 4096));
  hipLaunchKernelGGL(k_um_robin_fold, dim3(nb), dim3(kBlock), 0, s, g, T);
}

// SELL rows -> the stencil slots of a structured-topology mesh: all 27, or
// (half) the upper 14 (X zeroed first; a row's padding entries -- column r,
// value 0 -- add 0 to its centre; the lower entries of a half stencil are the
// neighbours' upper slots)
__global__ __launch_bounds__(kBlock) void k_um_to_stencil(int64_t nrow, const int64_t* __restrict__ soff,
                                                          const int* __restrict__ cols, const double* __restrict__ V,
                                                          int64_t s1, int64_t s2, int64_t nv, double* __restrict__ X,
                                                          int half) {
  for (int64_t r = blockIdx.x * (int64_t)kBlock + threadIdx.x; r < nrow; r += (int64_t)gridDim.x * kBlock) {
    const int64_t sl = r >> 6, lane = r & 63, so = soff[sl];
    const int wdt = (int)((soff[sl + 1] - so) >> 6);
    for (int k = 0; k < wdt; ++k) {
      const int64_t e = so + 64 * k + lane;
      const int64_t off = (int64_t)cols[e] - r;
      const int64_t dk = (off + s2 / 2 + s2) / s2 - 1;  // |di + s1 dj| < s2 / 2
      const int64_t rem = off - dk * s2;
      const int64_t dj = (rem + s1 / 2 + s1) / s1 - 1;  // |di| < s1 / 2
      const int64_t di = rem - dj * s1;
      const int q = (int)((di + 1) + 3 * (dj + 1) + 9 * (dk + 1));
      if (!half) X[(int64_t)q * nv + r] += V[e];
      else if (q >= 13) X[(int64_t)(q - 13) * nv + r] += V[e];
    }
  }
}

// A hexahedral mesh whose vertex and cell numbering is a box's: vertex v = i +
// N0 (j + N1 k), every cell the box cell of its first vertex in the tensor
// order l = a + 2b + 4c (from_rectilinear, a jittered / warped plate, an
// extruded gmsh mesh).  The coordinates can be anything.
static bool structured_topology(int dim, int64_t nv, int64_t nc, const int64_t* cells, int64_t* s1, int64_t* s2) {
  if (dim != 3 || nc < 1) return false;
  const int64_t N0 = cells[2] - cells[0], P = cells[4] - cells[0];
  if (cells[1] - cells[0] != 1 || N0 < 3 || P < 3 * N0 || P % N0 != 0 || nv % P != 0) return false;
  const int64_t N1 = P / N0, N2 = nv / P;
  if (N2 < 2 || nc != (N0 - 1) * (N1 - 1) * (N2 - 1)) return false;
  std::vector<char> seen((size_t)nv, 0);
  for (int64_t e = 0; e < nc; ++e) {
    const int64_t b = cells[e * 8];
    if (b < 0 || b >= nv) return false;
    const int64_t i = b % N0, j = (b / N0) % N1, k = b / P;
    if (i >= N0 - 1 || j >= N1 - 1 || k >= N2 - 1 || seen[(size_t)b]) return false;
    seen[(size_t)b] = 1;
    for (int l = 1; l < 8; ++l)
      if (cells[e * 8 + l] != b + (l & 1) + N0 * ((l >> 1) & 1) + P * (l >> 2)) return false;
  }
  *s1 = N0;
  *s2 = P;
  return true;
}

// ---- host: mesh analysis and device setup ----------------------------------------
#define UMC(x)                                                             \
  do {                                                                     \
    if ((x) != hipSuccess) {                                               \
      err = std::string("HIP error in unstructured setup: ") + #x;         \
      return 1;                                                            \
    }                                                                      \
  } while (0)

template <class T>
static int um_upload(UmDevice* d, const std::vector<T>& h, T** out, std::string& err) {
  void* p = nullptr;
  UMC(hipMalloc(&p, sizeof(T) * std::max<size_t>(1, h.size())));
  d->bufs.push_back(p);
  if (!h.empty()) UMC(hipMemcpy(p, h.data(), sizeof(T) * h.size(), hipMemcpyHostToDevice));
  *out = static_cast<T*>(p);
  return 0;
}

template <class T>
static int um_alloc(UmDevice* d, size_t n, T** out, std::string& err) {
  void* p = nullptr;
  UMC(hipMalloc(&p, sizeof(T) * std::max<size_t>(1, n)));
  d->bufs.push_back(p);
  *out = static_cast<T*>(p);
  return 0;
}

static void release(UmDevice* d, void* p) {
  auto it = std::find(d->bufs.begin(), d->bufs.end(), p);
  if (it != d->bufs.end()) {
    hipFree(p);
    d->bufs.erase(it);
  }
}

// boundary facets: local facets whose sorted vertex set occurs once; (cell, lf)
// in cell order
static int boundary_facets(int dim, int64_t nc, const int64_t* cells, std::vector<std::pair<int64_t, int>>& bf,
                           std::string& err) {
  const int nl = 1 << dim;
  struct F {
    int64_t v[4];
    int64_t cell;
    int lf;
  };
  const int nfv = nl / 2;
  std::vector<F> fs;
  fs.reserve((size_t)nc * 2 * dim);
  for (int64_t e = 0; e < nc; ++e)
    for (int lf = 0; lf < 2 * dim; ++lf) {
      F f{{-1, -1, -1, -1}, e, lf};
      int k = 0;
      for (int l = 0; l < nl; ++l)
        if (((l >> (lf >> 1)) & 1) == (lf & 1)) f.v[k++] = cells[e * nl + l];
      std::sort(f.v, f.v + nfv);
      fs.push_back(f);
    }
  auto key_less = [&](const F& a, const F& b) {
    for (int k = 0; k < nfv; ++k)
      if (a.v[k] != b.v[k]) return a.v[k] < b.v[k];
    return false;
  };
  auto key_eq = [&](const F& a, const F& b) {
    for (int k = 0; k < nfv; ++k)
      if (a.v[k] != b.v[k]) return false;
    return true;
  };
  std::sort(fs.begin(), fs.end(), [&](const F& a, const F& b) {
    if (key_less(a, b)) return true;
    if (key_less(b, a)) return false;
    return a.cell < b.cell;
  });
  bf.clear();
  for (size_t i = 0; i < fs.size();) {
    size_t j = i + 1;
    while (j < fs.size() && key_eq(fs[i], fs[j])) ++j;
    if (j - i == 1) bf.emplace_back(fs[i].cell, fs[i].lf);
    else if (j - i > 2) {
      err = "non-manifold mesh: a facet shared by more than two cells";
      return 1;
    }
    i = j;
  }
  std::sort(bf.begin(), bf.end());
  return 0;
}

static int n_threads() {
  const unsigned h = std::thread::hardware_concurrency();
  return (int)std::max(1u, std::min(16u, h ? h : 1u));
}

void um_free(UmDevice* d) {
  if (!d) return;
  for (void* p : d->bufs) hipFree(p);
  delete d;
}

int um_setup(int dim, int64_t nv, int64_t nrow, const double* xyz, int64_t nc, const int64_t* cells, UmGrid& g,
             UmDevice*& dev, hipStream_t s, std::string& err) {
  const int nl = 1 << dim;
  if (nrow < 1 || nrow > nv) {
    err = "unstructured setup: owned rows out of range";
    return 1;
  }
  dev = new UmDevice();
  UmDevice* d = dev;
  // -- boundary facets
  std::vector<std::pair<int64_t, int>> bf;
  if (boundary_facets(dim, nc, cells, bf, err)) return 1;
  const int64_t nf = (int64_t)bf.size();
  // -- vertex -> (cell, local vertex) incidences, cell order
  std::vector<int64_t> inc_off((size_t)nv + 1, 0), inc((size_t)nc * nl);
  for (int64_t k = 0; k < nc * nl; ++k) inc_off[(size_t)cells[k] + 1]++;
  for (int64_t v = 0; v < nv; ++v) inc_off[v + 1] += inc_off[v];
  {
    std::vector<int64_t> fill(inc_off.begin(), inc_off.end() - 1);
    for (int64_t e = 0; e < nc; ++e)
      for (int l = 0; l < nl; ++l) inc[(size_t)fill[(size_t)cells[e * nl + l]]++] = (e << 3) | l;
  }
  // -- sparsity pattern: the vertices of the cells around each vertex (sorted);
  // rows [0, nrow) only (a partition: its owned vertices, whose cells are all
  // local -- the ghost rows are never computed)
  const int nth = n_threads();
  std::vector<int> rnnz((size_t)nrow, 0);
  std::vector<std::vector<int>> part((size_t)nth);
  std::vector<int64_t> r0((size_t)nth + 1);
  for (int t = 0; t <= nth; ++t) r0[t] = nrow * t / nth;
  {
    std::vector<std::thread> th;
    for (int t = 0; t < nth; ++t)
      th.emplace_back([&, t]() {
        std::vector<int> buf;
        auto& out = part[(size_t)t];
        for (int64_t r = r0[t]; r < r0[t + 1]; ++r) {
          buf.clear();
          for (int64_t q = inc_off[r]; q < inc_off[r + 1]; ++q) {
            const int64_t e = inc[(size_t)q] >> 3;
            for (int j = 0; j < nl; ++j) buf.push_back((int)cells[e * nl + j]);
          }
          std::sort(buf.begin(), buf.end());
          buf.erase(std::unique(buf.begin(), buf.end()), buf.end());
          rnnz[(size_t)r] = (int)buf.size();
          out.insert(out.end(), buf.begin(), buf.end());
        }
      });
    for (auto& x : th) x.join();
  }
  // -- SELL-64 layout
  const int64_t nslice = (nrow + 63) / 64;
  std::vector<int64_t> soff((size_t)nslice + 1, 0);
  for (int64_t sl = 0; sl < nslice; ++sl) {
    int w = 0;
    for (int64_t r = sl * 64; r < std::min(nrow, sl * 64 + 64); ++r) w = std::max(w, rnnz[(size_t)r]);
    soff[(size_t)sl + 1] = soff[(size_t)sl] + 64 * (int64_t)w;
  }
  const int64_t nnz = soff[(size_t)nslice];
  std::vector<int> cols((size_t)nnz, 0);
  {
    std::vector<std::thread> th;
    for (int t = 0; t < nth; ++t)
      th.emplace_back([&, t]() {
        size_t pos = 0;
        const auto& src = part[(size_t)t];
        for (int64_t r = r0[t]; r < r0[t + 1]; ++r) {
          const int64_t sl = r >> 6, lane = r & 63;
          const int w = (int)((soff[(size_t)sl + 1] - soff[(size_t)sl]) >> 6);
          for (int k = 0; k < w; ++k)
            cols[(size_t)(soff[(size_t)sl] + 64 * k + lane)] = k < rnnz[(size_t)r] ? src[pos + k] : (int)r;
          pos += (size_t)rnnz[(size_t)r];
        }
      });
    for (auto& x : th) x.join();
  }
  // padding lanes of the last slice (rows >= nrow) keep column 0, value 0
  std::vector<std::vector<int>>().swap(part);
  d->nnz = nnz;
  // -- boundary facet data (host): incidences of the boundary rows
  const int nfv = nl / 2;
  std::vector<int> fcell((size_t)nf);
  std::vector<signed char> flf((size_t)nf);
  std::vector<int> boff((size_t)nv + 1, 0);
  for (int64_t f = 0; f < nf; ++f) {
    fcell[(size_t)f] = (int)bf[(size_t)f].first;
    flf[(size_t)f] = (signed char)bf[(size_t)f].second;
    const int64_t e = bf[(size_t)f].first;
    const int lf = bf[(size_t)f].second;
    for (int l = 0; l < nl; ++l)
      if (((l >> (lf >> 1)) & 1) == (lf & 1)) boff[(size_t)cells[e * nl + l] + 1]++;
  }
  for (int64_t v = 0; v < nv; ++v) boff[(size_t)v + 1] += boff[(size_t)v];
  std::vector<int> binc((size_t)boff[(size_t)nv]);
  {
    std::vector<int> fill(boff.begin(), boff.end() - 1);
    for (int64_t f = 0; f < nf; ++f) {
      const int64_t e = bf[(size_t)f].first;
      const int lf = bf[(size_t)f].second;
      int m = 0;
      for (int l = 0; l < nl; ++l)
        if (((l >> (lf >> 1)) & 1) == (lf & 1)) binc[(size_t)fill[(size_t)cells[e * nl + l]]++] = (int)(4 * f + m++);
    }
  }
  // (a partition's ghost layer has outer facets that are not on the domain
  // boundary; no owned row touches them, and the mask covers owned rows only)
  d->bmask.assign((size_t)nv, 0);
  d->nb = 0;
  for (int64_t v = 0; v < nrow; ++v)
    if (boff[(size_t)v + 1] > boff[(size_t)v]) {
      d->bmask[(size_t)v] = 1;
      d->nb++;
    }
  (void)nfv;
  // -- uploads
  std::vector<double> Xh[3];
  double* Xd[3];
  for (int a = 0; a < 3; ++a) {
    Xh[a].resize((size_t)nv);
    for (int64_t v = 0; v < nv; ++v) Xh[a][(size_t)v] = xyz[3 * v + a];
    if (um_upload(d, Xh[a], &Xd[a], err)) return 1;
    std::vector<double>().swap(Xh[a]);
  }
  std::vector<int> cell_h((size_t)nl * nc);
  for (int64_t e = 0; e < nc; ++e)
    for (int l = 0; l < nl; ++l) cell_h[(size_t)l * nc + e] = (int)cells[e * nl + l];
  int *cell_d, *cols_d, *rnnz_d, *fcell_d, *fv_d, *boff_d, *binc_d;
  int64_t *inc_off_d, *inc_d, *soff_d;
  signed char* flf_d;
  double *V, *M, *K, *bvec, *vdiag, *fw;
  if (um_upload(d, cell_h, &cell_d, err) || um_upload(d, cols, &cols_d, err) || um_upload(d, rnnz, &rnnz_d, err) ||
      um_upload(d, inc_off, &inc_off_d, err) || um_upload(d, inc, &inc_d, err) || um_upload(d, soff, &soff_d, err) ||
      um_upload(d, fcell, &fcell_d, err) || um_upload(d, flf, &flf_d, err) || um_upload(d, boff, &boff_d, err) ||
      um_upload(d, binc, &binc_d, err))
    return 1;
  std::vector<int>().swap(cell_h);
  std::vector<int>().swap(cols);
  std::vector<int64_t>().swap(inc);
  if (um_alloc(d, (size_t)nnz, &V, err) || um_alloc(d, (size_t)nnz, &M, err) || um_alloc(d, (size_t)nnz, &K, err) ||
      um_alloc(d, (size_t)nv, &bvec, err) || um_alloc(d, (size_t)nv, &vdiag, err) ||
      um_alloc(d, (size_t)nfv * nf, &fv_d, err) || um_alloc(d, (size_t)(dim == 2 ? 3 : 9) * nf, &fw, err))
    return 1;
  UMC(hipMemsetAsync(V, 0, sizeof(double) * (size_t)std::max<int64_t>(1, nnz), s));
  UMC(hipMemsetAsync(M, 0, sizeof(double) * (size_t)std::max<int64_t>(1, nnz), s));
  UMC(hipMemsetAsync(K, 0, sizeof(double) * (size_t)std::max<int64_t>(1, nnz), s));
  UMC(hipMemsetAsync(vdiag, 0, sizeof(double) * (size_t)nv, s));
  const double dt_alpha = g.dt_alpha;
  const dim3 bl(kBlock);
  const dim3 gr_v((unsigned)((nrow + kBlock - 1) / kBlock)), gr_f((unsigned)std::max<int64_t>(1, (nf + kBlock - 1) / kBlock));
  if (dim == 2) {
    hipLaunchKernelGGL((k_um_assemble<2>), gr_v, bl, 0, s, nrow, nc, cell_d, Xd[0], Xd[1], Xd[2], inc_off_d, inc_d,
                       soff_d, cols_d, rnnz_d, dt_alpha, V, M, K, bvec, vdiag);
    if (nf) hipLaunchKernelGGL((k_um_facet_setup<2>), gr_f, bl, 0, s, nf, nc, fcell_d, flf_d, cell_d, Xd[0], Xd[1],
                               Xd[2], fv_d, fw);
  } else {
    hipLaunchKernelGGL((k_um_assemble<3>), gr_v, bl, 0, s, nrow, nc, cell_d, Xd[0], Xd[1], Xd[2], inc_off_d, inc_d,
                       soff_d, cols_d, rnnz_d, dt_alpha, V, M, K, bvec, vdiag);
    if (nf) hipLaunchKernelGGL((k_um_facet_setup<3>), gr_f, bl, 0, s, nf, nc, fcell_d, flf_d, cell_d, Xd[0], Xd[1],
                               Xd[2], fv_d, fw);
  }
  UMC(hipGetLastError());
  // structured topology on one partition: J x from the half stencil (the
  // residual stays on SELL: its 27-slot M and K stencils measured no faster,
  // 1.03-1.14 vs 1.01 ms -- the boundary rows' facet quadrature bounds it --
  // and their half forms slower, 1.35 ms: the lower slots' re-reads a plane
  // apart miss L2)
  int64_t ss1 = 0, ss2 = 0, nbr = 0;
  double *V14 = nullptr, *J14 = nullptr, *M14 = nullptr, *K14 = nullptr;
  int64_t* brow_d = nullptr;
  // (32-bit element offsets into the 14 slot arrays: 14 nv * 8 B < 4 GiB)
  if (nrow == nv && nv * 14 * 8 < ((int64_t)1 << 32) && structured_topology(dim, nv, nc, cells, &ss1, &ss2)) {
    const size_t n14 = (size_t)14 * nv;
    if (um_alloc(d, n14, &V14, err) || um_alloc(d, n14, &J14, err) || um_alloc(d, n14, &M14, err) ||
        um_alloc(d, n14, &K14, err))
      return 1;
    for (double* X : {V14, M14, K14}) UMC(hipMemsetAsync(X, 0, sizeof(double) * n14, s));
    hipLaunchKernelGGL(k_um_to_stencil, gr_v, bl, 0, s, nrow, soff_d, cols_d, V, ss1, ss2, nv, V14, 1);
    hipLaunchKernelGGL(k_um_to_stencil, gr_v, bl, 0, s, nrow, soff_d, cols_d, M, ss1, ss2, nv, M14, 1);
    hipLaunchKernelGGL(k_um_to_stencil, gr_v, bl, 0, s, nrow, soff_d, cols_d, K, ss1, ss2, nv, K14, 1);
    UMC(hipGetLastError());
    UMC(hipMemcpyAsync(J14, V14, sizeof(double) * n14, hipMemcpyDeviceToDevice, s));
  }
  {  // the owned rows with boundary incidences (the Robin passes)
    std::vector<int64_t> brow;
    for (int64_t v = 0; v < nrow; ++v)
      if (boff[(size_t)v + 1] > boff[(size_t)v]) brow.push_back(v);
    nbr = (int64_t)brow.size();
    if (nbr > 0 && um_upload(d, brow, &brow_d, err)) return 1;
  }
  UMC(hipStreamSynchronize(s));
  // setup-only arrays
  for (void* p : {(void*)Xd[0], (void*)Xd[1], (void*)Xd[2], (void*)cell_d, (void*)rnnz_d, (void*)inc_off_d,
                  (void*)inc_d, (void*)fcell_d, (void*)flf_d})
    release(d, p);
  g.dim = dim;
  g.nv = nv;
  g.nrow = nrow;
  g.nc = nc;
  g.nf = nf;
  g.nslice = nslice;
  g.soff = soff_d;
  g.cols = cols_d;
  g.V = V;
  g.M = M;
  g.K = K;
  g.bvec = bvec;
  g.vdiag = vdiag;
  g.V14 = V14;
  g.J14 = J14;
  g.M14 = M14;
  g.K14 = K14;
  g.brow = brow_d;
  g.nbr = nbr;
  g.s1 = ss1;
  g.s2 = ss2;
  g.fv = fv_d;
  g.fw = fw;
  g.boff = boff_d;
  g.binc = binc_d;
  return 0;
}
#undef UMC

// ---- host: recursive coordinate bisection of the cells ----------------------------
// Splits the cell set along the axis of largest centroid extent so that the two
// halves hold cells in proportion to the part counts they receive (any number of
// parts, not only powers of two).  Deterministic: ties broken by cell index.
// Replaces the graph partitioner dolfinx calls when a mesh is distributed
// (create_mesh with the default partitioner, gmshio.read_from_msh at
// ThermoViscoProblem.py:27-28).
static void rcb_split(const std::vector<double>& cen, std::vector<int64_t>& idx, int64_t lo, int64_t hi, int p0,
                      int np, int* part) {
  if (np == 1) {
    for (int64_t k = lo; k < hi; ++k) part[idx[(size_t)k]] = p0;
    return;
  }
  double mn[3] = {1e300, 1e300, 1e300}, mx[3] = {-1e300, -1e300, -1e300};
  for (int64_t k = lo; k < hi; ++k)
    for (int a = 0; a < 3; ++a) {
      const double v = cen[3 * (size_t)idx[(size_t)k] + a];
      mn[a] = std::min(mn[a], v);
      mx[a] = std::max(mx[a], v);
    }
  int ax = 0;
  for (int a = 1; a < 3; ++a)
    if (mx[a] - mn[a] > mx[ax] - mn[ax]) ax = a;
  const int nl = np / 2;
  const int64_t mid = lo + (int64_t)((double)(hi - lo) * nl / np + 0.5);
  auto less = [&](int64_t x, int64_t y) {
    const double vx = cen[3 * (size_t)x + ax], vy = cen[3 * (size_t)y + ax];
    return vx < vy || (vx == vy && x < y);
  };
  std::nth_element(idx.begin() + lo, idx.begin() + mid, idx.begin() + hi, less);
  rcb_split(cen, idx, lo, mid, p0, nl, part);
  rcb_split(cen, idx, mid, hi, p0 + nl, np - nl, part);
}

int um_rcb(int dim, int64_t nv, const double* xyz, int64_t nc, const int64_t* cells, int n_parts, int* part,
           std::string& err) {
  if (n_parts < 1 || n_parts > nc) {
    err = "n_parts must be in [1, n_cells]";
    return 1;
  }
  const int nl = 1 << dim;
  std::vector<double> cen((size_t)3 * nc, 0.0);
  for (int64_t e = 0; e < nc; ++e)
    for (int l = 0; l < nl; ++l) {
      const int64_t v = cells[(size_t)e * nl + l];
      if (v < 0 || v >= nv) {
        err = "cell vertex index out of range";
        return 1;
      }
      for (int a = 0; a < 3; ++a) cen[3 * (size_t)e + a] += xyz[3 * (size_t)v + a] / nl;
    }
  std::vector<int64_t> idx((size_t)nc);
  for (int64_t e = 0; e < nc; ++e) idx[(size_t)e] = e;
  rcb_split(cen, idx, 0, nc, 0, n_parts, part);
  return 0;
}

}  // namespace tv
