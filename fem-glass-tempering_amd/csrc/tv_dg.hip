// DG1 (discontinuous Q1 / P1) symmetric interior-penalty operators on
// rectilinear grids, gfx950.
//
// Replaces, for fe_config["T"] = DG (ThermoViscoProblem.py:308-325):
//   * the FFCx cell kernel (mass + alpha grad.grad, :295-300),
//   * the FFCx interior-facet kernel of the SIPG terms
//        dt*alpha('+') * ( p/h('+') jump(v,n).jump(T,n)
//                          - avg(grad v).jump(T,n) - jump(v,n).avg(grad T) ) dS
//     with p = 5 (:313) and h = CellDiameter (:314),
//   * the FFCx exterior-facet kernel of the Robin terms (:302-304),
// and their Jacobians, plus the PETSc MatMult / diagonal on the assembled matrix.
//
// Rectilinear cells make every term a tensor product of per-axis 2x2 (cell) or
// 2x4 (face, normal direction) matrices with the tangential 1D masses, which
// the kernel evaluates on the fly from the per-axis cell lengths.  '+' of an
// interior facet is the lower-index cell (the cell below along the facet
// normal).  One thread owns one cell and produces its 2^d rows; dof layout is
// component-major [local dof][cell] so the 2^d loads of a wave are coalesced.
#include "tv_internal.h"

namespace tv {
namespace {

enum { MODE_RES = 0, MODE_JAC = 1 };

__device__ constexpr double kGX[3] = {0.11270166537925831148, 0.5, 0.88729833462074168852};
__device__ constexpr double kGW[3] = {5.0 / 18.0, 8.0 / 18.0, 5.0 / 18.0};

template <int DIM>
struct Ax {
  static constexpr int NA = DIM;       // active storage axes
  static constexpr int NL = 1 << DIM;  // local dofs per cell
  __device__ static constexpr int axis(int k) { return DIM == 2 ? (k == 0 ? 0 : 2) : k; }
};

__device__ __forceinline__ double gfun(const DgGrid& g, double T) {
  const double T2 = T * T;
  return g.a_rad * (T2 * T2 - g.T_amb4) + g.a_conv * (T - g.T_amb);
}
__device__ __forceinline__ double dgfun(const DgGrid& g, double T) { return g.a_rad * 4.0 * (T * T * T) + g.a_conv; }

__device__ __forceinline__ double mloc(double h, int a, int b) { return h * (a == b ? (1.0 / 3.0) : (1.0 / 6.0)); }
__device__ __forceinline__ double kloc(double h, int a, int b) { return (a == b ? 1.0 : -1.0) / h; }

template <int DIM, int MODE, bool FUSEP>
__global__ __launch_bounds__(kBlock) void k_dg_cells(DgGrid g, const double* __restrict__ T,
                                                     const double* __restrict__ in0, const double* in1,
                                                     double* __restrict__ out, double* pout,
                                                     const PcgState* __restrict__ st,
                                                     double* __restrict__ partials) {
  using A = Ax<DIM>;
  constexpr int NL = A::NL;
  __shared__ double red[kBlock / kWave];
  if (FUSEP && st->done) return;
  const int64_t ncell = (int64_t)g.c0 * g.c1 * g.c2;
  const int64_t cstride = ncell;  // component stride
  const int64_t cid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool ok = cid < ncell;
  const int ci[3] = {ok ? (int)(cid % g.c0) : 0, ok ? (int)((cid / g.c0) % g.c1) : 0,
                     ok ? (int)(cid / ((int64_t)g.c0 * g.c1)) : 0};
  const int cn[3] = {g.c0, g.c1, g.c2};
  const int64_t cst[3] = {1, g.c0, (int64_t)g.c0 * g.c1};

  double bcoef = 0.0;
  bool first = false;
  const double* pold = in1;
  if (FUSEP) {
    const int it = st->it;
    first = (it == 0);
    bcoef = first ? 0.0 : st->beta / st->betaold;
    if (!(it & 1)) { pold = pout; pout = const_cast<double*>(in1); }
  }
  auto ld = [&](int64_t c, int l) -> double {  // input value (p for FUSEP)
    const int64_t o = (int64_t)l * cstride + c;
    double v = in0[o];
    if (FUSEP && !first) v = v + bcoef * pold[o];
    return v;
  };
  double h[3] = {1.0, 1.0, 1.0};
#pragma unroll
  for (int k = 0; k < A::NA; ++k) h[A::axis(k)] = g.h[A::axis(k)][ci[A::axis(k)]];
  double hd2 = 0.0;
#pragma unroll
  for (int k = 0; k < A::NA; ++k) hd2 += h[A::axis(k)] * h[A::axis(k)];

  double x[NL], m[NL], y[NL];
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    x[l] = ok ? ld(cid, l) : 0.0;
    m[l] = 0.0;
    if (MODE == MODE_RES && ok) m[l] = x[l] - in1[(int64_t)l * cstride + cid] - g.dt_f;
    y[l] = 0.0;
  }
  // ---- cell term: M m + dt alpha K x (tensor products of 2x2 blocks) ----
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    double acc = 0.0;
#pragma unroll
    for (int q = 0; q < NL; ++q) {
      double mm = 1.0;
      double kk = 0.0;
#pragma unroll
      for (int k = 0; k < A::NA; ++k) {
        const int a = (l >> k) & 1, b = (q >> k) & 1;
        const double hk = h[A::axis(k)];
        double prod = kloc(hk, a, b);
#pragma unroll
        for (int e = 0; e < A::NA; ++e)
          if (e != k) prod *= mloc(h[A::axis(e)], (l >> e) & 1, (q >> e) & 1);
        kk += prod;
        mm *= mloc(hk, a, b);
      }
      const double mass_in = (MODE == MODE_RES) ? m[q] : x[q];
      acc += mm * mass_in + g.dt_alpha * kk * x[q];
    }
    y[l] = acc;
  }
  // ---- faces ----
#pragma unroll
  for (int k = 0; k < A::NA; ++k) {
    const int ax = A::axis(k);
#pragma unroll
    for (int side = 0; side < 2; ++side) {
      const int nbi = ci[ax] + (side ? 1 : -1);
      const bool interior = nbi >= 0 && nbi < cn[ax];
      if (interior) {
        const int64_t nb = cid + (side ? cst[ax] : -cst[ax]);
        double xn[NL];
#pragma unroll
        for (int l = 0; l < NL; ++l) xn[l] = ok ? ld(nb, l) : 0.0;
        // L = lower cell, R = upper cell along ax; '+' = L
        const double hL = side ? h[ax] : g.h[ax][ok ? nbi : 0];
        const double hR = side ? g.h[ax][ok ? nbi : 0] : h[ax];
        double hdL2 = hd2 - h[ax] * h[ax] + hL * hL;
        const double pen = g.penalty / sqrt(hdL2);
        // J = [0, 1, -1, 0], G = [-1/(2hL), 1/(2hL), -1/(2hR), 1/(2hR)] over (L0, L1, R0, R1)
        const double Jv[4] = {0.0, 1.0, -1.0, 0.0};
        const double Gv[4] = {-0.5 / hL, 0.5 / hL, -0.5 / hR, 0.5 / hR};
#pragma unroll
        for (int l = 0; l < NL; ++l) {
          const int bl = (l >> k) & 1;
          const int row = side ? bl : 2 + bl;  // this cell is L on its upper face, R on its lower face
          double acc = 0.0;
#pragma unroll
          for (int q = 0; q < NL; ++q) {
            const int bq = (q >> k) & 1;
            double mt = 1.0;
#pragma unroll
            for (int e = 0; e < A::NA; ++e)
              if (e != k) mt *= mloc(h[A::axis(e)], (l >> e) & 1, (q >> e) & 1);
            const int colown = side ? bq : 2 + bq;
            const int colnb = side ? 2 + bq : bq;
            const double a_own = pen * Jv[row] * Jv[colown] - Gv[row] * Jv[colown] - Jv[row] * Gv[colown];
            const double a_nb = pen * Jv[row] * Jv[colnb] - Gv[row] * Jv[colnb] - Jv[row] * Gv[colnb];
            acc += mt * (a_own * x[q] + a_nb * xn[q]);
          }
          y[l] += g.dt_alpha * acc;
        }
      } else if (g.bnd[ax][side]) {
        // Robin facet on the physical boundary: face dofs have bit k == side
        double Tl[NL];
#pragma unroll
        for (int l = 0; l < NL; ++l) {
          if (MODE == MODE_RES) Tl[l] = x[l];
          else Tl[l] = ok ? T[(int64_t)l * cstride + cid] : 0.0;
        }
        constexpr int NT = A::NA - 1;  // tangential active axes
        constexpr int NQ = NT == 0 ? 1 : (NT == 1 ? 3 : 9);
        double acc[NL];
#pragma unroll
        for (int l = 0; l < NL; ++l) acc[l] = 0.0;
#pragma unroll
        for (int qq = 0; qq < NQ; ++qq) {
          // tangential coordinates / weights
          double w = 1.0;
          double xi_t[3] = {0.0, 0.0, 0.0};
          int t = 0;
#pragma unroll
          for (int e = 0; e < A::NA; ++e) {
            if (e == k) continue;
            const int qi = (t == 0) ? (qq % 3) : (qq / 3);
            xi_t[e] = kGX[qi];
            w *= kGW[qi] * h[A::axis(e)];
            ++t;
          }
          double phi[NL];
          double Th = 0.0, Ph = 0.0;
#pragma unroll
          for (int l = 0; l < NL; ++l) {
            double f = (((l >> k) & 1) == side) ? 1.0 : 0.0;
#pragma unroll
            for (int e = 0; e < A::NA; ++e)
              if (e != k) f *= ((l >> e) & 1) ? xi_t[e] : 1.0 - xi_t[e];
            phi[l] = f;
            Th += f * Tl[l];
            Ph += f * x[l];
          }
          const double gv = (MODE == MODE_RES) ? gfun(g, Th) : dgfun(g, Th) * Ph;
#pragma unroll
          for (int l = 0; l < NL; ++l) acc[l] += w * gv * phi[l];
        }
#pragma unroll
        for (int l = 0; l < NL; ++l) y[l] += g.dt * acc[l];
      }
    }
  }
  const bool owned = ok && ci[2] >= g.k_begin && ci[2] < g.k_end;
  double dot = 0.0;
  if (ok) {
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      const int64_t o = (int64_t)l * cstride + cid;
      if (FUSEP) pout[o] = x[l];
      if (owned) {
        out[o] = y[l];
        dot += x[l] * y[l];
      }
    }
  }
  if (MODE == MODE_JAC && partials != nullptr) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) dot += __shfl_xor(dot, off, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = dot;
    __syncthreads();
    if (threadIdx.x == 0) partials[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
  }
}

// diag(J) by applying the operator to unit vectors of the cell (NL applies).
template <int DIM>
__global__ __launch_bounds__(kBlock) void k_dg_diag(DgGrid g, const double* __restrict__ T,
                                                    double* __restrict__ out, int invert) {
  using A = Ax<DIM>;
  constexpr int NL = A::NL;
  const int64_t ncell = (int64_t)g.c0 * g.c1 * g.c2;
  const int64_t cid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (cid >= ncell) return;
  const int ci[3] = {(int)(cid % g.c0), (int)((cid / g.c0) % g.c1), (int)(cid / ((int64_t)g.c0 * g.c1))};
  const int cn[3] = {g.c0, g.c1, g.c2};
  double h[3] = {1.0, 1.0, 1.0};
#pragma unroll
  for (int k = 0; k < A::NA; ++k) h[A::axis(k)] = g.h[A::axis(k)][ci[A::axis(k)]];
  double hd2 = 0.0;
#pragma unroll
  for (int k = 0; k < A::NA; ++k) hd2 += h[A::axis(k)] * h[A::axis(k)];
  double Tl[NL];
#pragma unroll
  for (int l = 0; l < NL; ++l) Tl[l] = T[(int64_t)l * ncell + cid];
#pragma unroll
  for (int l = 0; l < NL; ++l) {
    double mm = 1.0, kk = 0.0;
#pragma unroll
    for (int k = 0; k < A::NA; ++k) {
      const int a = (l >> k) & 1;
      double prod = kloc(h[A::axis(k)], a, a);
#pragma unroll
      for (int e = 0; e < A::NA; ++e)
        if (e != k) prod *= mloc(h[A::axis(e)], (l >> e) & 1, (l >> e) & 1);
      kk += prod;
      mm *= mloc(h[A::axis(k)], a, a);
    }
    double d = mm + g.dt_alpha * kk;
#pragma unroll
    for (int k = 0; k < A::NA; ++k) {
      const int ax = A::axis(k);
      const int bl = (l >> k) & 1;
#pragma unroll
      for (int side = 0; side < 2; ++side) {
        const int nbi = ci[ax] + (side ? 1 : -1);
        double mt = 1.0;
#pragma unroll
        for (int e = 0; e < A::NA; ++e)
          if (e != k) mt *= mloc(h[A::axis(e)], (l >> e) & 1, (l >> e) & 1);
        if (nbi >= 0 && nbi < cn[ax]) {
          const double hL = side ? h[ax] : g.h[ax][nbi];
          const double hR = side ? g.h[ax][nbi] : h[ax];
          const double pen = g.penalty / sqrt(hd2 - h[ax] * h[ax] + hL * hL);
          const double Jv[4] = {0.0, 1.0, -1.0, 0.0};
          const double Gv[4] = {-0.5 / hL, 0.5 / hL, -0.5 / hR, 0.5 / hR};
          const int row = side ? bl : 2 + bl;
          d += g.dt_alpha * mt * (pen * Jv[row] * Jv[row] - 2.0 * Gv[row] * Jv[row]);
        } else if (g.bnd[ax][side] && bl == side) {
          constexpr int NT = A::NA - 1;
          constexpr int NQ = NT == 0 ? 1 : (NT == 1 ? 3 : 9);
          double acc = 0.0;
#pragma unroll
          for (int qq = 0; qq < NQ; ++qq) {
            double w = 1.0;
            double xi_t[3] = {0.0, 0.0, 0.0};
            int t = 0;
#pragma unroll
            for (int e = 0; e < A::NA; ++e) {
              if (e == k) continue;
              const int qi = (t == 0) ? (qq % 3) : (qq / 3);
              xi_t[e] = kGX[qi];
              w *= kGW[qi] * h[A::axis(e)];
              ++t;
            }
            double Th = 0.0, phil = 0.0;
#pragma unroll
            for (int q = 0; q < NL; ++q) {
              double f = (((q >> k) & 1) == side) ? 1.0 : 0.0;
#pragma unroll
              for (int e = 0; e < A::NA; ++e)
                if (e != k) f *= ((q >> e) & 1) ? xi_t[e] : 1.0 - xi_t[e];
              Th += f * Tl[q];
              if (q == l) phil = f;
            }
            acc += w * dgfun(g, Th) * phil * phil;
          }
          d += g.dt * acc;
        }
      }
    }
    out[(int64_t)l * ncell + cid] = invert ? 1.0 / d : d;
  }
}

int dg_dim(const DgGrid& g) { return g.deg2 ? 1 : (g.deg1 ? 2 : 3); }

template <int MODE, bool FUSEP>
void launch_cells(const DgGrid& g, const double* T, const double* in0, const double* in1, double* out,
                  double* pout, const PcgState* st, double* partials, hipStream_t s, int* nparts) {
  const int64_t ncell = (int64_t)g.c0 * g.c1 * g.c2;
  const int blocks = (int)((ncell + kBlock - 1) / kBlock);
  if (nparts) *nparts = blocks;
  if (blocks <= 0) return;
  switch (dg_dim(g)) {
    case 1:
      hipLaunchKernelGGL((k_dg_cells<1, MODE, FUSEP>), dim3(blocks), dim3(kBlock), 0, s, g, T, in0, in1, out, pout,
                         st, partials);
      break;
    case 2:
      hipLaunchKernelGGL((k_dg_cells<2, MODE, FUSEP>), dim3(blocks), dim3(kBlock), 0, s, g, T, in0, in1, out, pout,
                         st, partials);
      break;
    default:
      hipLaunchKernelGGL((k_dg_cells<3, MODE, FUSEP>), dim3(blocks), dim3(kBlock), 0, s, g, T, in0, in1, out, pout,
                         st, partials);
  }
}

}  // namespace

void launch_dg_residual(const DgGrid& g, const double* T, const double* Tp, double* F, hipStream_t s) {
  launch_cells<MODE_RES, false>(g, T, T, Tp, F, nullptr, nullptr, nullptr, s, nullptr);
}

void launch_dg_japply(const DgGrid& g, const double* T, const double* x, double* y, double* partials,
                      int* n_partials, hipStream_t s) {
  launch_cells<MODE_JAC, false>(g, T, x, nullptr, y, nullptr, nullptr, partials, s, n_partials);
}

void launch_dg_japply_fused(const DgGrid& g, const double* T, const double* z, double* pA, double* pB, double* w,
                            const PcgState* st, double* partials, int* n_partials, hipStream_t s) {
  launch_cells<MODE_JAC, true>(g, T, z, pA, w, pB, st, partials, s, n_partials);
}

void launch_dg_diag(const DgGrid& g, const double* T, double* dinv, int invert, hipStream_t s) {
  const int64_t ncell = (int64_t)g.c0 * g.c1 * g.c2;
  const int blocks = (int)((ncell + kBlock - 1) / kBlock);
  if (blocks <= 0) return;
  switch (dg_dim(g)) {
    case 1: hipLaunchKernelGGL(k_dg_diag<1>, dim3(blocks), dim3(kBlock), 0, s, g, T, dinv, invert); break;
    case 2: hipLaunchKernelGGL(k_dg_diag<2>, dim3(blocks), dim3(kBlock), 0, s, g, T, dinv, invert); break;
    default: hipLaunchKernelGGL(k_dg_diag<3>, dim3(blocks), dim3(kBlock), 0, s, g, T, dinv, invert);
  }
}

}  // namespace tv
