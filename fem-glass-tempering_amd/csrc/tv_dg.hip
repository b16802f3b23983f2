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
#include <algorithm>
#include <cstdlib>

#include "tv_device.h"

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

// dof addressing of a cell layer k (see DgGrid): dof of component l of the
// cell at in-layer index ij (= i + c0 j) is base + l stride + ij
struct DgAddr {
  int64_t base, stride;
};
__device__ __forceinline__ DgAddr dg_layer(const DgGrid& g, int k) {
  const int64_t pc = (int64_t)g.c0 * g.c1;
  if (k < g.k_begin) return {g.gofs[0], pc};
  if (k >= g.k_end) return {g.gofs[1], pc};
  return {(int64_t)(k - g.k_begin) * pc, g.own};
}

__device__ __forceinline__ double gfun(const DgGrid& g, double T) {
  const double T2 = T * T;
  return g.a_rad * (T2 * T2 - g.T_amb4) + g.a_conv * (T - g.T_amb);
}
__device__ __forceinline__ double dgfun(const DgGrid& g, double T) { return g.a_rad * 4.0 * (T * T * T) + g.a_conv; }

__device__ __forceinline__ double mloc(double h, int a, int b) { return h * (a == b ? (1.0 / 3.0) : (1.0 / 6.0)); }
__device__ __forceinline__ double kloc(double h, int a, int b) { return (a == b ? 1.0 : -1.0) / h; }
// SIPG penalty / sqrt(q) without the FP64 sqrt + divide sequences (~25
// instructions each, a third of the tile kernels' per-cell VALU count): v_rsq_f64
// refined by two Newton steps (relative error ~1e-16, not bitwise the IEEE quotient)
__device__ __forceinline__ double pen_rsq(double penalty, double q) {
  double r = __builtin_amdgcn_rsq(q);
  r = r * (1.5 - (0.5 * q) * (r * r));
  r = r * (1.5 - (0.5 * q) * (r * r));
  return penalty * r;
}

// v <- (M_e (x) I) v along storage axis e (local bit e), M_e = h [1/3 1/6; 1/6 1/3]
__device__ __forceinline__ void mass_axis(double (&v)[8], int e, double h) {
  const double d = h * (1.0 / 3.0), o = h * (1.0 / 6.0);
#pragma unroll
  for (int l = 0; l < 8; ++l)
    if (!((l >> e) & 1)) {
      const double a = v[l], b = v[l | (1 << e)];
      v[l] = d * a + o * b;
      v[l | (1 << e)] = o * a + d * b;
    }
}
// out <- (K_e (x) I) v, K_e = (1/h) [1 -1; -1 1]; ih = 1/h
__device__ __forceinline__ void stiff_axis(const double (&v)[8], double (&out)[8], int e, double ih) {
#pragma unroll
  for (int l = 0; l < 8; ++l)
    if (!((l >> e) & 1)) {
      const double dlt = (v[l] - v[l | (1 << e)]) * ih;
      out[l] = dlt;
      out[l | (1 << e)] = -dlt;
    }
}

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
  const int64_t cid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool ok = cid < ncell;
  const int ci[3] = {ok ? (int)(cid % g.c0) : 0, ok ? (int)((cid / g.c0) % g.c1) : 0,
                     ok ? (int)(cid / ((int64_t)g.c0 * g.c1)) : 0};
  const int cn[3] = {g.c0, g.c1, g.c2};
  const int64_t cst[3] = {1, g.c0, (int64_t)g.c0 * g.c1};
  const int64_t ij = (int64_t)ci[0] + (int64_t)g.c0 * ci[1];  // in-layer index
  const DgAddr ac = dg_layer(g, ci[2]);

  double bcoef = 0.0;
  bool first = false;
  const double* pold = in1;
  if (FUSEP) {
    const int it = st->it;
    first = (it == 0);
    bcoef = first ? 0.0 : st->beta / st->betaold;
    if (!(it & 1)) { pold = pout; pout = const_cast<double*>(in1); }
  }
  auto ld = [&](const DgAddr& a, int64_t q, int l) -> double {  // input value (p for FUSEP)
    const int64_t o = a.base + (int64_t)l * a.stride + q;
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
    x[l] = ok ? ld(ac, ij, l) : 0.0;
    m[l] = 0.0;
    if (MODE == MODE_RES && ok) m[l] = x[l] - in1[ac.base + (int64_t)l * ac.stride + ij] - g.dt_f;
    y[l] = 0.0;
  }
  // ---- cell term: M m + dt alpha K x (tensor products of 2x2 blocks) ----
  if constexpr (DIM == 3 && MODE == MODE_RES) {
    // the residual (no tile kernel for it): sum-factorised, ~0.2 kflop per cell
    // instead of the 8 x 8 entry-by-entry product below (kept for the Jacobian
    // reference path the tile kernel is tested against)
    double A[8], B[8], C[8], D[8], U[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) {
      A[l] = m[l];
      C[l] = x[l];
    }
    const double ih[3] = {g.ih[0][ci[0]], g.ih[1][ci[1]], g.ih[2][ci[2]]};
    mass_axis(A, 0, h[0]); mass_axis(A, 1, h[1]); mass_axis(A, 2, h[2]);  // Mz My Mx m
    stiff_axis(x, B, 0, ih[0]); mass_axis(B, 1, h[1]); mass_axis(B, 2, h[2]);  // Mz My Kx x
    mass_axis(C, 0, h[0]);                                                   // Mx x
    stiff_axis(C, D, 1, ih[1]); mass_axis(D, 2, h[2]);                       // Mz Ky Mx x
    mass_axis(C, 1, h[1]);
    stiff_axis(C, U, 2, ih[2]);                                              // Kz My Mx x
#pragma unroll
    for (int l = 0; l < 8; ++l) y[l] = A[l] + g.dt_alpha * ((B[l] + D[l]) + U[l]);
  } else {
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
        // the neighbour: another layer along axis 2, else the same layer
        const DgAddr an = (ax == 2) ? dg_layer(g, nbi) : ac;
        const int64_t ijn = (ax == 2) ? ij : ij + (side ? cst[ax] : -cst[ax]);
        double xn[NL];
#pragma unroll
        for (int l = 0; l < NL; ++l) xn[l] = ok ? ld(an, ijn, l) : 0.0;
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
          else Tl[l] = ok ? T[ac.base + (int64_t)l * ac.stride + ij] : 0.0;
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
      const int64_t o = ac.base + (int64_t)l * ac.stride + ij;
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


// ---- cell-block Jacobi (the multigrid smoother of DG1 level 0) ----------------------
// B_c = the 8 x 8 diagonal block of J(T) for cell c (its own dofs): the cell
// term, the SIPG self-couplings of its interior facets and its Robin facets.
// On a box cell every term is a Kronecker product of 1D 2 x 2 matrices,
//   B_c = Mx (x) My (x) Mz + dt alpha (Ax (x) My (x) Mz + Mx (x) Ay (x) Mz + Mx (x) My (x) Az),
// A_k = the 1D stiffness + the SIPG self terms of the two facets along k (+ the
// Robin term on a boundary facet), so B_c^-1 is applied by fast diagonalisation:
// A_k V_k = M_k V_k L_k per axis (2 x 2, closed form), B_c^-1 =
// (Vx (x) Vy (x) Vz) (I + dt alpha (Lx + Ly + Lz))^-1 (Vx (x) Vy (x) Vz)^T -- no
// per-cell storage.  The one approximation: the Robin facet weight dg(T) is
// taken constant over a facet (the mean of its 4 nodal values, gface below; the
// 3 x 3 Gauss sum of the operator varies it), which keeps the block separable.
// The smoother only has to be symmetric positive definite and close to B_c.

// per boundary facet: mean of dg(T) over its 4 nodes; layout per axis k (the two
// other axes a < b): [side][i_a][i_b], axes concatenated (gface_offsets)
__device__ __forceinline__ void gface_offsets(const DgGrid& g, int64_t (&off)[4]) {
  off[0] = 0;
  off[1] = off[0] + 2 * (int64_t)g.c1 * g.c2;
  off[2] = off[1] + 2 * (int64_t)g.c0 * g.c2;
  off[3] = off[2] + 2 * (int64_t)g.c0 * g.c1;
}

__global__ __launch_bounds__(kBlock) void k_dg_gface(DgGrid g, const double* __restrict__ T,
                                                     double* __restrict__ gface) {
  int64_t off[4];
  gface_offsets(g, off);
  const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (t >= off[3]) return;
  const int k = t < off[1] ? 0 : (t < off[2] ? 1 : 2);
  const int cn[3] = {g.c0, g.c1, g.c2};
  const int ea = k == 0 ? 1 : 0, eb = k == 2 ? 1 : 2;
  const int64_t r = t - off[k];
  const int ib = (int)(r % cn[eb]), ia = (int)((r / cn[eb]) % cn[ea]), side = (int)(r / ((int64_t)cn[ea] * cn[eb]));
  int ci[3];
  ci[k] = side ? cn[k] - 1 : 0;
  ci[ea] = ia;
  ci[eb] = ib;
  const DgAddr a = dg_layer(g, ci[2]);  // a slab's layers (DgGrid)
  const int64_t ij = ci[0] + (int64_t)g.c0 * ci[1];
  double acc = 0.0;
#pragma unroll
  for (int l = 0; l < 8; ++l)
    if (((l >> k) & 1) == side) acc += dgfun(g, T[a.base + (int64_t)l * a.stride + ij]);
  gface[t] = 0.25 * acc;
}

// Reciprocal and reciprocal square root for the smoother's arithmetic:
// v_rcp_f64 / v_rsq_f64 and one Newton step (relative error ~1e-12 or better,
// ~5 instructions instead of the ~10-25 of an IEEE divide / sqrt).  The block
// smoother only has to be a fixed SPD operator: the same cell always gets the
// same V and Lambda, before and after the coarse correction.
__device__ __forceinline__ double frcp(double x) {
  const double r = __builtin_amdgcn_rcp(x);
  return r * (2.0 - x * r);
}
__device__ __forceinline__ double frsq(double x) {
  const double r = __builtin_amdgcn_rsq(x);
  return r * (1.5 - (0.5 * x) * (r * r));
}

// A v = lambda M v for M = h/6 [[2, 1], [1, 2]] and symmetric A: with S = M^-1/2
// = [[p, q], [q, p]], one Jacobi rotation diagonalises C = S A S; V = S J.
// ih = 1 / h.
__device__ __forceinline__ void fdm2(double ih, double a00, double a01, double a11, double (&V)[4], double (&lam)[2]) {
  const double s0 = (2.0 * ih) * frsq(2.0 * ih), s1 = 1.7320508075688772 * s0;  // sqrt(2 / h), sqrt(6 / h)
  const double p = 0.5 * (s0 + s1), q = 0.5 * (s0 - s1);
  const double b00 = a00 * p + a01 * q, b01 = a00 * q + a01 * p;
  const double b10 = a01 * p + a11 * q, b11 = a01 * q + a11 * p;
  const double c00 = p * b00 + q * b10, c01 = p * b01 + q * b11, c11 = q * b01 + p * b11;
  double t = 0.0, cs = 1.0, sn = 0.0;
  if (c01 != 0.0) {
    const double tau = (c11 - c00) * frcp(2.0 * c01);
    const double q1 = 1.0 + tau * tau;
    t = (tau >= 0.0 ? 1.0 : -1.0) * frcp(fabs(tau) + q1 * frsq(q1));
    cs = frsq(1.0 + t * t);
    sn = t * cs;
  }
  lam[0] = c00 - t * c01;
  lam[1] = c11 + t * c01;
  // V = S [[cs, sn], [-sn, cs]], row-major V[row * 2 + col]
  V[0] = p * cs - q * sn;
  V[1] = p * sn + q * cs;
  V[2] = q * cs - p * sn;
  V[3] = q * sn + p * cs;
}

// y = B_c^-1 v for cell cid (fast diagonalisation, see above)
__device__ __forceinline__ void fdm_mul(const DgGrid& g, const double* __restrict__ gface, int64_t cid,
                                        const double (&v)[8], double (&y)[8]) {
  const int cn[3] = {g.c0, g.c1, g.c2};
  const int ci[3] = {(int)(cid % g.c0), (int)((cid / g.c0) % g.c1), (int)(cid / ((int64_t)g.c0 * g.c1))};
  // every table value first (the neighbours' lengths at clamped indices):
  // loaded where used, under the facet branches, each waited for the load
  // before it -- six dependent round trips per cell
  double h[3], ihk[3], hnb[3][2];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    h[k] = g.h[k][ci[k]];
    ihk[k] = g.ih[k][ci[k]];
    hnb[k][0] = g.h[k][max(ci[k] - 1, 0)];
    hnb[k][1] = g.h[k][min(ci[k] + 1, cn[k] - 1)];
  }
  const double hd2 = h[0] * h[0] + h[1] * h[1] + h[2] * h[2];
  int64_t off[4];
  gface_offsets(g, off);
  double V[3][4], lam[3][2];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const double hk = h[k], ih = ihk[k];
    double a00 = ih, a01 = -ih, a11 = ih;  // 1D stiffness
    const int ea = k == 0 ? 1 : 0, eb = k == 2 ? 1 : 2;
#pragma unroll
    for (int side = 0; side < 2; ++side) {
      const int nbi = ci[k] + (side ? 1 : -1);
      if (nbi >= 0 && nbi < cn[k]) {  // SIPG self terms of the facet (rows of k_dg_diag)
        const double hn = hnb[k][side];
        const double pen = g.penalty * frsq(side ? hd2 : hd2 - hk * hk + hn * hn);
        a01 += 0.5 * ih;
        if (side) a11 += pen - ih;
        else a00 += pen - ih;
      } else if (g.bnd[k][side]) {  // Robin: dt dg e e^T (x) M (x) M = dt alpha (dg / alpha) ...
        const double gw = gface[off[k] + ((int64_t)side * cn[ea] + ci[ea]) * cn[eb] + ci[eb]];
        const double r = g.dt / g.dt_alpha * gw;
        if (side) a11 += r;
        else a00 += r;
      }
    }
    fdm2(ih, a00, a01, a11, V[k], lam[k]);
  }
  double u[8];
#pragma unroll
  for (int l = 0; l < 8; ++l) u[l] = v[l];
  // u <- (Vx (x) Vy (x) Vz)^T u
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int l = 0; l < 8; ++l)
      if (!((l >> k) & 1)) {
        const int m = l | (1 << k);
        const double u0 = u[l], u1 = u[m];
        u[l] = V[k][0] * u0 + V[k][2] * u1;
        u[m] = V[k][1] * u0 + V[k][3] * u1;
      }
#pragma unroll
  for (int l = 0; l < 8; ++l)
    u[l] *= frcp(1.0 + g.dt_alpha * (lam[0][l & 1] + lam[1][(l >> 1) & 1] + lam[2][(l >> 2) & 1]));
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int l = 0; l < 8; ++l)
      if (!((l >> k) & 1)) {
        const int m = l | (1 << k);
        const double u0 = u[l], u1 = u[m];
        u[l] = V[k][0] * u0 + V[k][1] * u1;
        u[m] = V[k][2] * u0 + V[k][3] * u1;
      }
#pragma unroll
  for (int l = 0; l < 8; ++l) y[l] = u[l];
}

// ---------------------------------------------------------------------------
// 3D Jacobian apply on an (x-segment x rows) tile of cells marching through a
// chunk of planes: the SIPG J x of k_dg_cells<3, MODE_JAC>, restructured for
// the hardware.
//   * lane = cell along storage axis 0 (62 outputs per wave, lanes 0 / 63 are
//     the x-halo cells); x-neighbour values come from the next / previous lane
//     (DPP wave shifts), not from memory;
//   * wave = row along axis `ra`; R compute waves plus one halo wave above and
//     below exchange their 8 values per cell through LDS (one barrier);
//   * the neighbours along the march axis `pa` are the previous / next plane,
//     held in registers (plane L + 1 is loaded while plane L is computed);
//   * every operator term is sum-factorised: 2x2 mass / stiffness factors per
//     axis for the cell term; for each interior facet the 4-column normal SIPG
//     matrix, then the two tangential 2x2 masses (~0.5 kflop per cell, not ~3).
// FUSEP: x = p = z + beta/betaold p_old formed on the fly and stored (as
// k_dg_cells); out = w on owned cells; one p.w partial per workgroup.
// (Fusing the DG multigrid post-smoothing -- prolongation, J x, cell-block
// solve and the (z.z, z.r) records -- into this kernel measured slower than the
// three separate kernels at C5: 195 us vs 187 us; the epilogue runs at 2 waves
// per SIMD with 254 VGPRs.)
// ---------------------------------------------------------------------------
constexpr int kDgRows = 6;  // + 2 halo waves: 512 threads, up to 256 VGPRs (no spills)
constexpr int kDgRowsHL = 8;  // HL: 8 computing waves, the edge waves also load the halo rows
constexpr int dg_rows(bool hl) { return hl ? kDgRowsHL : kDgRows; }

// HL (halo loads): no halo waves -- all 8 waves compute a row and waves 0 / 7
// also load the rows above / below the tile (plane L + 1 in flight during step
// L, formed into the slab's halo slots at the top of step L + 1): 8 output
// rows per 8 waves instead of 6.
// RA: the row axis (1 or 2) as a template parameter, so every k == ra / pa
// test and ci[] / cn[] index in the unrolled facet loop resolves at compile time
template <bool FUSEP, bool HL, int RA>
__global__ __launch_bounds__(512) void k_dg_tile(DgGrid g, const double* __restrict__ T,
                                                 const double* __restrict__ in0, const double* in1,
                                                 double* __restrict__ out, double* pout,
                                                 const PcgState* __restrict__ st, double* __restrict__ partials,
                                                 int nseg, int qchunk, int nch, RedTail rt) {
  constexpr int ra = RA;
  stamp_start(rt);
  constexpr int R = dg_rows(HL);
  constexpr int NW = HL ? R : R + 2;  // waves per workgroup (512 threads either way)
  __shared__ double sX[2][R + 2][8][kWave];  // double-buffered plane slab: one barrier per plane
  __shared__ double red[NW];
  if (st != nullptr && st->done) return;  // uniform over the grid
  const int pa = 3 - ra;
  const int cn[3] = {g.c0, g.c1, g.c2};
  const int npl = cn[pa];
  // chunk fastest: the chunks of one column of tiles share their boundary
  // planes and land on one XCD (contiguous range after the remap)
  const int b = xcd_remap((int)blockIdx.x, (int)gridDim.x);
  // (segment fastest, as the CG march: the same at C5, measured)
  const int chunk = b % nch;
  const int t = b / nch;
  const int seg = t % nseg;
  const int rb = t / nseg;
  const int q0 = chunk * qchunk, q1 = min(q0 + qchunk, npl);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & (kWave - 1);
  const int r = HL ? rb * R + wave : rb * R - 1 + wave;  // row along ra (!HL: waves 0 and R + 1 are halo rows)
  const int slot = HL ? wave + 1 : wave;                   // the row's slot in the slab
  const int i = seg * kSeg - 1 + lane;
  const bool valid = i >= 0 && i < g.c0 && r >= 0 && r < cn[ra];
  const bool compute = HL || (wave >= 1 && wave <= R);
  const bool writer = compute && valid && lane >= 1 && lane <= kSeg;
  // HL: the halo row this wave loads (wave 0: the row below the tile, wave R - 1: above)
  const int rh = wave == 0 ? r - 1 : r + 1;
  // dof addressing (DgAddr) of the cell of row rr in plane L: the cell layer is
  // the row (ra = 2) or the plane (ra = 1).  The row and the plane are
  // wave-uniform (clamped into the grid; out-of-grid loads and stores are
  // masked by the caller), so the layer base and stride stay scalar and only
  // the in-layer index is per lane (a lane-masked row made them per-lane
  // 64-bit values: 256 VGPRs and 140 B of scratch per lane, fused matvec 97
  // -> 153 us at C5)
  const int rcl = min(max(r, 0), cn[ra] - 1), rhcl = min(max(rh, 0), cn[ra] - 1);
  auto cell_addr = [&](int ii, int rr, int L, int64_t& q) -> DgAddr {
    const int Lc = min(max(L, 0), npl - 1);
    q = (int64_t)ii + (int64_t)g.c0 * (ra == 2 ? Lc : rr);
    return dg_layer(g, ra == 2 ? rr : Lc);
  };
  const bool hvalid = HL && (wave == 0 || wave == R - 1) && i >= 0 && i < g.c0 && rh >= 0 && rh < cn[ra];
  const int hslot = wave == 0 ? 0 : R + 1;

  double bcoef = 0.0;
  bool first = false;
  const double* pold = in1;
  if (FUSEP) {
    const int it = st->it;
    first = (it == 0);
    bcoef = first ? 0.0 : st->beta / st->betaold;
    if (!(it & 1)) { pold = pout; pout = const_cast<double*>(in1); }
  }
  // raw loads of this lane's cell in plane L (0 outside the grid), then the
  // input values (p = z + b p_old for FUSEP)
  auto fetch = [&](int L, double (&rz)[8], double (&ro)[8]) {
    const bool ok = valid && L >= 0 && L < npl;
    int64_t q;
    const DgAddr a = cell_addr(valid ? i : 0, rcl, L, q);
#pragma unroll
    for (int l = 0; l < 8; ++l) {
      const int64_t o = a.base + (int64_t)l * a.stride + q;
      rz[l] = ok ? in0[o] : 0.0;
      ro[l] = (FUSEP && !first && ok) ? pold[o] : 0.0;
    }
  };
  auto form = [&](const double (&rz)[8], const double (&ro)[8], double (&v)[8]) {
#pragma unroll
    for (int l = 0; l < 8; ++l) v[l] = FUSEP ? rz[l] + bcoef * ro[l] : rz[l];
  };
  double hz[8], ho[8];  // HL: raw loads of the halo row of plane L + 1, in flight during step L
  auto hfetch = [&](int L) {
    const bool ok = hvalid && L >= 0 && L < npl;
    int64_t q;
    const DgAddr a = cell_addr(hvalid ? i : 0, rhcl, L, q);
#pragma unroll
    for (int l = 0; l < 8; ++l) {
      const int64_t o = a.base + (int64_t)l * a.stride + q;
      hz[l] = ok ? in0[o] : 0.0;
      ho[l] = (FUSEP && !first && ok) ? pold[o] : 0.0;
    }
  };
  if (HL) hfetch(q0);
  // cell lengths: the x axis per lane and the row axis per wave do not change
  // along the march (loaded once; the x neighbours' by DPP); the march axis'
  // per plane by scalar loads.  Vector loads of the tables inside the march
  // made every plane wait for the plane prefetch too (vmcnt counts in order)
  const int icl = min(max(i, 0), g.c0 - 1);
  const double h0 = g.h[0][icl], ih0 = g.ih[0][icl];
  const int rlo = max(rcl - 1, 0), rhi = min(rcl + 1, cn[ra] - 1);
  const double hr = kld(g.h[ra], rcl), ihr = kld(g.ih[ra], rcl);
  const double hr_lo = kld(g.h[ra], rlo), ihr_lo = kld(g.ih[ra], rlo);
  const double hr_hi = kld(g.h[ra], rhi), ihr_hi = kld(g.ih[ra], rhi);
  double xl[8], x[8], xu[8];  // planes L - 1, L, L + 1
  double rz[8], ro[8];        // raw loads of plane L + 2, in flight during step L
  {  // prologue: the loads of the first three planes in flight together
    double az[8], ao[8], bz[8], bo[8];
    fetch(q0 - 1, az, ao);
    fetch(q0, bz, bo);
    fetch(q0 + 1, rz, ro);
    form(az, ao, xl);
    form(bz, bo, x);
    form(rz, ro, xu);
  }
  double dot = 0.0;
  for (int L = q0; L < q1; ++L) {
    fetch(L + 2, rz, ro);
    const int sb = L & 1;
#pragma unroll
    for (int l = 0; l < 8; ++l) sX[sb][slot][l][lane] = x[l];
    if (HL && (wave == 0 || wave == R - 1)) {  // wave-uniform
#pragma unroll
      for (int l = 0; l < 8; ++l) sX[sb][hslot][l][lane] = FUSEP ? hz[l] + bcoef * ho[l] : hz[l];
      hfetch(L + 1);
    }
    int64_t cq;
    const DgAddr ca = cell_addr(valid ? i : 0, rcl, L, cq);
    if (FUSEP && writer) {
#pragma unroll
      for (int l = 0; l < 8; ++l) pout[ca.base + (int64_t)l * ca.stride + cq] = x[l];
    }
    __syncthreads();
    if (compute) {  // wave-uniform: every lane runs the DPP exchanges below; stores are masked
      int ci[3];
      ci[0] = valid ? i : 0;
      ci[ra] = valid ? r : 0;
      ci[pa] = L;
      double h[3], ih[3];
      h[0] = h0;
      ih[0] = ih0;
      h[ra] = hr;
      ih[ra] = ihr;
      h[pa] = kld(g.h[pa], L);
      ih[pa] = kld(g.ih[pa], L);
      const double hd2 = h[0] * h[0] + h[1] * h[1] + h[2] * h[2];
      const double pen_up = pen_rsq(g.penalty, hd2);  // upper facets: this cell is '+'
      double y[8];
      // ---- cell term: Mz(My Mx x + da (My Kx x + Ky Mx x)) + da Kz (My Mx x) ----
      {
        double A[8], B[8], AK[8];
#pragma unroll
        for (int l = 0; l < 8; ++l) A[l] = x[l];
        stiff_axis(x, B, 0, ih[0]);  // Kx x
        mass_axis(A, 0, h[0]);       // Mx x
        stiff_axis(A, AK, 1, ih[1]); // Ky Mx x
        mass_axis(A, 1, h[1]);       // My Mx x
        mass_axis(B, 1, h[1]);       // My Kx x
        double S[8];
#pragma unroll
        for (int l = 0; l < 8; ++l) S[l] = A[l] + g.dt_alpha * (B[l] + AK[l]);
        mass_axis(S, 2, h[2]);
        double KA[8];
        stiff_axis(A, KA, 2, ih[2]);
#pragma unroll
        for (int l = 0; l < 8; ++l) y[l] = S[l] + g.dt_alpha * KA[l];
      }
      // ---- facets ----
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int e1 = (k == 0) ? 1 : 0, e2 = (k == 2) ? 1 : 2;  // tangential axes
        double Us[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};  // both facets along k: one pair of tangential masses
#pragma unroll
        for (int side = 0; side < 2; ++side) {
          const int nbi = ci[k] + (side ? 1 : -1);
          const bool interior = valid && nbi >= 0 && nbi < cn[k];
          double xn[8], hn, ihn;  // the neighbour's values and lengths along k
          if (k == 0) {  // lane +- 1 (all lanes)
#pragma unroll
            for (int l = 0; l < 8; ++l) xn[l] = side ? shl1(x[l]) : shr1(x[l]);
            hn = side ? shl1(h0) : shr1(h0);
            ihn = side ? shl1(ih0) : shr1(ih0);
          } else if (k == ra) {
#pragma unroll
            for (int l = 0; l < 8; ++l) xn[l] = sX[sb][slot + (side ? 1 : -1)][l][lane];
            hn = side ? hr_hi : hr_lo;
            ihn = side ? ihr_hi : ihr_lo;
          } else {
#pragma unroll
            for (int l = 0; l < 8; ++l) xn[l] = side ? xu[l] : xl[l];
            const int Ln = min(max(L + (side ? 1 : -1), 0), npl - 1);
            hn = kld(g.h[pa], Ln);
            ihn = kld(g.ih[pa], Ln);
          }
          if (interior) {
            // SIPG facet rows, '+' = L = lower cell: with J = (0, 1, -1, 0) and
            // G = (-gL, gL, -gR, gR), g = 1/(2h), the 4x4 normal matrix
            // pen J J^T - G J^T - J G^T reduces per tangential dof pair to the
            // jump j = x_L1 - x_R0 and the normal differences d = x_1 - x_0 of
            // both cells; then the tangential masses (they commute)
            const double gO = 0.5 * ih[k], gN = 0.5 * ihn;
            double U[8];
            if (side) {  // upper facet: this cell is L, the neighbour R
              const double pen = pen_up;
#pragma unroll
              for (int tt = 0; tt < 4; ++tt) {
                const int l0 = ((tt & 1) << e1) | ((tt >> 1) << e2), l1 = l0 | (1 << k);
                const double j = x[l1] - xn[l0], dO = x[l1] - x[l0], dN = xn[l1] - xn[l0];
                U[l0] = gO * j;
                U[l1] = (pen - gO) * j - gO * dO - gN * dN;
              }
            } else {  // lower facet: this cell is R, the neighbour L ('+', its lengths set the penalty)
              const double pen = pen_rsq(g.penalty, hd2 - h[k] * h[k] + hn * hn);
#pragma unroll
              for (int tt = 0; tt < 4; ++tt) {
                const int l0 = ((tt & 1) << e1) | ((tt >> 1) << e2), l1 = l0 | (1 << k);
                const double j = xn[l1] - x[l0], dO = x[l1] - x[l0], dN = xn[l1] - xn[l0];
                U[l1] = -gO * j;
                U[l0] = (gO - pen) * j + gO * dO + gN * dN;
              }
            }
#pragma unroll
            for (int l = 0; l < 8; ++l) Us[l] += U[l];
          } else if (valid && g.bnd[k][side]) {
            // Robin facet Jacobian on the physical boundary (3x3 Gauss, as
            // k_dg_cells): only the 4 dofs on the facet (bit k == side) are nonzero there
            double Tf[4], Xf[4], acc[4];
#pragma unroll
            for (int f = 0; f < 4; ++f) {
              const int l = (side << k) | ((f & 1) << e1) | ((f >> 1) << e2);
              Tf[f] = T[ca.base + (int64_t)l * ca.stride + cq];
              Xf[f] = x[l];
              acc[f] = 0.0;
            }
#pragma unroll
            for (int qq = 0; qq < 9; ++qq) {
              const double s1 = kGX[qq % 3], s2 = kGX[qq / 3];
              const double w = (kGW[qq % 3] * h[e1]) * (kGW[qq / 3] * h[e2]);
              const double phi[4] = {(1.0 - s1) * (1.0 - s2), s1 * (1.0 - s2), (1.0 - s1) * s2, s1 * s2};
              double Th = 0.0, Ph = 0.0;
#pragma unroll
              for (int f = 0; f < 4; ++f) {
                Th += phi[f] * Tf[f];
                Ph += phi[f] * Xf[f];
              }
              const double gv = dgfun(g, Th) * Ph;
#pragma unroll
              for (int f = 0; f < 4; ++f) acc[f] += w * gv * phi[f];
            }
#pragma unroll
            for (int f = 0; f < 4; ++f) y[(side << k) | ((f & 1) << e1) | ((f >> 1) << e2)] += g.dt * acc[f];
          }
        }
        mass_axis(Us, e1, h[e1]);
        mass_axis(Us, e2, h[e2]);
#pragma unroll
        for (int l = 0; l < 8; ++l) y[l] += g.dt_alpha * Us[l];
      }
      if (writer && ci[2] >= g.k_begin && ci[2] < g.k_end) {
#pragma unroll
        for (int l = 0; l < 8; ++l) {
          out[ca.base + (int64_t)l * ca.stride + cq] = y[l];
          dot += x[l] * y[l];
        }
      }
    }
#pragma unroll
    for (int l = 0; l < 8; ++l) {
      xl[l] = x[l];
      x[l] = xu[l];
    }
    form(rz, ro, xu);
  }
  if (partials != nullptr) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) dot += __shfl_xor(dot, off, 64);
    if (lane == 0) red[wave] = dot;
    __syncthreads();
    if (threadIdx.x == 0) {
      double sacc = 0.0;
      for (int w = 0; w < NW; ++w) sacc += red[w];
      store_partial(&partials[blockIdx.x], sacc);
    }
    fused_reduce_tail<1>(rt, (int)gridDim.x);  // p.w over all tiles (+ KSPCG logic)
  }
}

struct DgTile {
  int nseg, ra, qchunk, nch, blocks;
};
DgTile dg_tile_plan(const DgGrid& g) {
  const int qmax = std::max(1, g.tile_chunk);  // planes marched per workgroup (default 5)
  DgTile p{};
  p.nseg = (g.c0 + kSeg - 1) / kSeg;
  p.ra = (g.c2 >= g.c1) ? 2 : 1;  // rows along the longer of axes 1 / 2, march along the other
  const int nr = (p.ra == 2) ? g.c2 : g.c1, npl = (p.ra == 2) ? g.c1 : g.c2;
  const int rows = dg_rows(true);
  const int nrb = (nr + rows - 1) / rows;
  p.nch = (npl + qmax - 1) / qmax;
  p.qchunk = (npl + p.nch - 1) / p.nch;
  p.nch = (npl + p.qchunk - 1) / p.qchunk;
  p.blocks = p.nseg * nrb * p.nch;
  return p;
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
  const DgAddr ac = dg_layer(g, ci[2]);
  const int64_t ij = (int64_t)ci[0] + (int64_t)g.c0 * ci[1];
  double Tl[NL];
#pragma unroll
  for (int l = 0; l < NL; ++l) Tl[l] = T[ac.base + (int64_t)l * ac.stride + ij];
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
    out[ac.base + (int64_t)l * ac.stride + ij] = invert ? 1.0 / d : d;
  }
}

// level >= 1 style smoothing step on DG: MODE 0 x = omega B^-1 b ; MODE 1 x += omega B^-1 (b - w)
// The block-smoother kernels run over the OWNED cells: dof (l, c) at l own + c
// (DgGrid: one partition owns every cell, a slab its own layers, which come
// first); fdm_mul takes the local cell index c + k_begin c0 c1.
template <int MODE>
__global__ __launch_bounds__(kBlock) void k_dg_bsmooth(DgGrid g, const PcgState* __restrict__ st,
                                                       const double* __restrict__ b, const double* __restrict__ w,
                                                       const double* __restrict__ gface, double omega,
                                                       double* __restrict__ x) {
  const int64_t ncell = g.own, c_loc = (int64_t)g.k_begin * g.c0 * g.c1;
  if (st != nullptr && st->done) return;
  for (int64_t c = blockIdx.x * (int64_t)kBlock + threadIdx.x; c < ncell; c += (int64_t)gridDim.x * kBlock) {
    double v[8], y[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) v[l] = MODE ? b[l * ncell + c] - w[l * ncell + c] : b[l * ncell + c];
    fdm_mul(g, gface, c + c_loc, v, y);
#pragma unroll
    for (int l = 0; l < 8; ++l) x[l * ncell + c] = MODE ? x[l * ncell + c] + omega * y[l] : omega * y[l];
  }
}

// KSPCG update with the explicit residual for the DG multigrid: r <- r - a w,
// dx <- dx + a p, x0 <- omega B^-1 r (INIT: dx <- 0, x0 <- omega B^-1 r)
// dx moves in pairs of iterations as in k_mg_update: DXU (odd iterations)
// dx <- (dx + a_prev p_prev) + a p, FIRST (iteration 1) assigns it, so the
// init pass leaves dx alone (launch_mg_dx_finish ends the solve)
template <bool INIT, bool DXU = false, bool FIRST = false>
__global__ __launch_bounds__(kBlock) void k_dg_bupdate(DgGrid g, const PcgState* __restrict__ st,
                                                       const double* __restrict__ pA, const double* __restrict__ pB,
                                                       const double* __restrict__ w, const double* __restrict__ gface,
                                                       double omega, double* __restrict__ r, double* __restrict__ dx,
                                                       double* __restrict__ x0, int it_host) {
  const int64_t ncell = g.own, c_loc = (int64_t)g.k_begin * g.c0 * g.c1;  // owned cells
  if (st->done) return;
  const double a = INIT ? 0.0 : st->a;
  const double ap = DXU ? st->a_prev : 0.0;
  const double* __restrict__ p = (it_host & 1) ? pB : pA;
  const double* __restrict__ pp = (it_host & 1) ? pA : pB;
  for (int64_t c = blockIdx.x * (int64_t)kBlock + threadIdx.x; c < ncell; c += (int64_t)gridDim.x * kBlock) {
    // every load of the cell before the first store (a store to r, then the
    // next copy's load from r: the compiler cannot prove them apart, so each
    // load waited for the store and the loads before it)
    double v[8], y[8], wv[8], dv[8], ppv[8], pv[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) {
      const int64_t o = l * ncell + c;
      v[l] = r[o];
      if (!INIT) wv[l] = __builtin_nontemporal_load(&w[o]);
      if (DXU) {
        dv[l] = FIRST ? 0.0 : __builtin_nontemporal_load(&dx[o]);
        ppv[l] = __builtin_nontemporal_load(&pp[o]);
        pv[l] = __builtin_nontemporal_load(&p[o]);
      }
    }
#pragma unroll
    for (int l = 0; l < 8; ++l) {
      const int64_t o = l * ncell + c;
      if (!INIT) {
        v[l] -= a * wv[l];
        r[o] = v[l];
        if (DXU) __builtin_nontemporal_store((dv[l] + ap * ppv[l]) + a * pv[l], &dx[o]);
      }
    }
    fdm_mul(g, gface, c + c_loc, v, y);
#pragma unroll
    for (int l = 0; l < 8; ++l) x0[l * ncell + c] = omega * y[l];
  }
}

// post-smoothing of DG level 0: z <- x0 + omega B^-1 (r - w); (z.z, z.r)
// records and the KSPCG logic in the reduction tail
__global__ __launch_bounds__(kBlock) void k_dg_bpost(DgGrid g, const PcgState* __restrict__ st,
                                                     const double* __restrict__ x0, const double* __restrict__ r,
                                                     const double* __restrict__ w, const double* __restrict__ gface,
                                                     double omega, double* __restrict__ z,
                                                     double* __restrict__ partials, RedTail rt) {
  const int64_t ncell = g.own, c_loc = (int64_t)g.k_begin * g.c0 * g.c1;  // owned cells
  __shared__ double red[2][kBlock / kWave];
  if (st->done) return;
  double acc[2] = {0.0, 0.0};
  for (int64_t c = blockIdx.x * (int64_t)kBlock + threadIdx.x; c < ncell; c += (int64_t)gridDim.x * kBlock) {
    // x0 loaded with r and w, before the smoother's table loads (it was
    // loaded after them: one more round trip per cell)
    double v[8], y[8], rr[8], xv[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) {
      rr[l] = r[l * ncell + c];
      v[l] = rr[l] - __builtin_nontemporal_load(&w[l * ncell + c]);  // w and x0: not read again
      xv[l] = __builtin_nontemporal_load(&x0[l * ncell + c]);
    }
    fdm_mul(g, gface, c + c_loc, v, y);
#pragma unroll
    for (int l = 0; l < 8; ++l) {
      const double zz = xv[l] + omega * y[l];
      z[l * ncell + c] = zz;
      acc[0] += zz * zz;
      acc[1] += zz * rr[l];
    }
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const double sw = wave_sum64(acc[q]);
    if (lane == 0) red[q][wave] = sw;
  }
  __syncthreads();
  if (threadIdx.x < 2)
    store_partial(&partials[(int64_t)blockIdx.x * 2 + threadIdx.x],
                  (red[threadIdx.x][0] + red[threadIdx.x][1]) + (red[threadIdx.x][2] + red[threadIdx.x][3]));
  fused_reduce_tail<2>(rt, gridDim.x);
}

int dg_vblocks(int64_t ncell) { return (int)std::max<int64_t>(1, std::min<int64_t>((ncell + kBlock - 1) / kBlock, 1024)); }

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

static bool dg_tiled(const DgGrid& g) { return g.tile && dg_dim(g) == 3; }  // 3D Jacobian: k_dg_tile

template <bool FUSEP>
static bool launch_tile(const DgGrid& g, const double* T, const double* in0, const double* in1, double* out,
                        double* pout, const PcgState* st, double* partials, int* n_partials, hipStream_t s,
                        const RedTail* tail = nullptr) {
  const DgTile p = dg_tile_plan(g);
  if (n_partials) *n_partials = p.blocks;
  if (p.blocks <= 0) return false;
  RedTail rt{};
  if (tail && partials) rt = *tail;
#define TV_DG_TILE(HLV, RAV)                                                                                  \
  hipLaunchKernelGGL((k_dg_tile<FUSEP, HLV, RAV>), dim3(p.blocks), dim3(512), 0, s, g, T, in0, in1, out, pout, st, \
                     partials, p.nseg, p.qchunk, p.nch, rt)
  // HL: 8 computing waves whose edge waves load the halo rows (the round-1
  // layout of 6 computing + 2 halo waves measured slower: J x 82 vs 64 us)
  if (p.ra == 2) TV_DG_TILE(true, 2);
  else TV_DG_TILE(true, 1);
#undef TV_DG_TILE
  return rt.counter != nullptr;
}

int dg_num_blocks(const DgGrid& g) {
  const int64_t ncell = (int64_t)g.c0 * g.c1 * g.c2;
  const int cells = (int)((ncell + kBlock - 1) / kBlock);
  return std::max(cells, dg_tile_plan(g).blocks);
}

void launch_dg_japply(const DgGrid& g, const double* T, const double* x, double* y, double* partials,
                      int* n_partials, hipStream_t s, const PcgState* st) {
  if (dg_tiled(g)) {
    launch_tile<false>(g, T, x, nullptr, y, nullptr, st, partials, n_partials, s);
    return;
  }
  launch_cells<MODE_JAC, false>(g, T, x, nullptr, y, nullptr, nullptr, partials, s, n_partials);
}

bool launch_dg_japply_fused(const DgGrid& g, const double* T, const double* z, double* pA, double* pB, double* w,
                            const PcgState* st, double* partials, int* n_partials, hipStream_t s,
                            const RedTail* tail) {
  if (dg_tiled(g)) return launch_tile<true>(g, T, z, pA, w, pB, st, partials, n_partials, s, tail);
  launch_cells<MODE_JAC, true>(g, T, z, pA, w, pB, st, partials, s, n_partials);
  return false;
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

int64_t dg_gface_size(const DgGrid& g) {
  return 2 * ((int64_t)g.c1 * g.c2 + (int64_t)g.c0 * g.c2 + (int64_t)g.c0 * g.c1);
}

void launch_dg_gface(const DgGrid& g, const double* T, double* gface, hipStream_t s) {
  const int64_t n = dg_gface_size(g);
  hipLaunchKernelGGL(k_dg_gface, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, g, T, gface);
}

void launch_dg_bsmooth(const DgGrid& g, const PcgState* st, const double* b, const double* w, const double* gface,
                       double omega, double* x, int mode, hipStream_t s) {
  const int nb = dg_vblocks(g.own);
  if (mode == 0) hipLaunchKernelGGL(k_dg_bsmooth<0>, dim3(nb), dim3(kBlock), 0, s, g, st, b, w, gface, omega, x);
  else hipLaunchKernelGGL(k_dg_bsmooth<1>, dim3(nb), dim3(kBlock), 0, s, g, st, b, w, gface, omega, x);
}

void launch_dg_bupdate(const DgGrid& g, const PcgState* st, const double* pA, const double* pB, const double* w,
                       const double* gface, double omega, double* r, double* dx, double* x0, int it_host, int init,
                       hipStream_t s) {
  const int nb = dg_vblocks(g.own);
#define TV_DGU(I, D, F) \
  hipLaunchKernelGGL((k_dg_bupdate<I, D, F>), dim3(nb), dim3(kBlock), 0, s, g, st, pA, pB, w, gface, omega, r, dx, x0, \
                     it_host)
  if (init) TV_DGU(true, false, false);
  else if (it_host == 1) TV_DGU(false, true, true);
  else if (it_host & 1) TV_DGU(false, true, false);
  else TV_DGU(false, false, false);
#undef TV_DGU
}

int launch_dg_bpost(const DgGrid& g, const PcgState* st, const double* x0, const double* r, const double* w,
                    const double* gface, double omega, double* z, double* partials, const RedTail* tail, hipStream_t s) {
  const RedTail rt = tail ? *tail : RedTail{};
  const int nb = dg_vblocks(g.own);
  hipLaunchKernelGGL(k_dg_bpost, dim3(nb), dim3(kBlock), 0, s, g, st, x0, r, w, gface, omega, z, partials, rt);
  return nb;
}

}  // namespace tv
