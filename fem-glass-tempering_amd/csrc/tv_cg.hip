// CG1 (Q1 hexahedra / P1 intervals) matrix-free operators on rectilinear grids,
// gfx950.
//
// Replaces, for the temperature space of ThermoViscoProblem (T family CG):
//   * the FFCx cell kernel of F dx (ThermoViscoProblem.py:295-300) and of its
//     Jacobian, driven by dolfinx assemble_vector / assemble_matrix, and
//   * the FFCx exterior-facet kernels of the Robin radiation + convection terms
//     (ThermoViscoProblem.py:302-304) and their Jacobian,
//   * PETSc MatMult / MatGetDiagonal on the assembled AIJ Jacobian.
//
// On a rectilinear grid the assembled Q1 operator factorises exactly:
//     M = Mz (x) My (x) Mx,
//     K = Mz (x) My (x) Kx + Mz (x) Ky (x) Mx + Kz (x) My (x) Mx
// with the assembled 1D P1 mass / stiffness (tridiagonal, per-node coefficients
// in CgGrid::coef).  The Robin facet integrals are evaluated per boundary node
// with 3x3 Gauss points per facet (exact for the degree-5-per-direction
// T^4 v and T^3 phi_i phi_j integrands).
//
// Execution shape (MI355X): one wavefront = one x-row segment of 64 nodes at
// fixed (j, k).  Each lane gathers its 3x3 (j, k)-column neighbourhood (9
// coalesced loads per wave-row, L1/L2-served for the neighbouring rows), folds
// the y and z directions in registers (sum factorisation: 34 FMA), and takes
// the x-neighbour partial sums from the adjacent lanes with DPP wave_shr /
// wave_shl (no LDS, no barriers).  Lanes 1..62 produce output.  The four waves
// of a workgroup take four consecutive j-rows so the j-neighbour rows are
// shared in L1.
#include <algorithm>
#include <cstdlib>

#include "tv_stencil.h"


#include <cstdio>
#include <vector>

namespace tv {
namespace {


// Raw buffer access (32-bit byte offsets against an SGPR descriptor).  The
// hardware range check returns 0 for loads and drops stores at offsets past
// the buffer, so out-of-domain neighbours and non-owned outputs are masked by
// an out-of-range offset (kBadOff) instead of branches.
using buf_t = __amdgpu_buffer_rsrc_t;
using b64v = unsigned int __attribute__((ext_vector_type(2)));
constexpr uint32_t kBadOff = 0x40000000u;  // > any buffer the march path accepts (host guard)
__device__ __forceinline__ buf_t mk_rsrc(const void* p, uint32_t bytes) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  void* q = (void*)(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(q, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
__device__ __forceinline__ double bload(buf_t r, uint32_t off) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 0));
}
__device__ __forceinline__ void bstore(buf_t r, uint32_t off, double v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(b64v, v), r, (int)off, 0, 0);
}

__device__ __forceinline__ double uniform(double v) {  // wave-uniform value -> SGPR pair
  const int lo = __builtin_amdgcn_readfirstlane(__double2loint(v));
  const int hi = __builtin_amdgcn_readfirstlane(__double2hiint(v));
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}


// ---------------------------------------------------------------------------
// Row-segment stencil kernel.
//   MODE_RES : out = F(T; Tp)  (in0 = T, in1 = Tp)
//   MODE_JAC : out = J(T) x    (in0 = x)                 [FUSEP = false]
//              p = z + beta/betaold p_old, out = J(T) p  (in0 = z, in1 = p_old -> pout)
//              (PETSc KSPCG "p <- z + b p" fused with MatMult, plus partial p.w)
// ---------------------------------------------------------------------------
template <int DIM, int MODE, bool FUSEP>
__global__ __launch_bounds__(kBlock) void k_cg_rows(CgGrid g, const double* __restrict__ T,
                                                    const double* __restrict__ in0,
                                                    const double* in1,
                                                    double* __restrict__ out, double* pout,
                                                    const PcgState* __restrict__ st,
                                                    double* __restrict__ partials, int nseg, int kfirst,
                                                    int nplanes, int wmode) {
  constexpr bool D1 = (DIM <= 2);  // storage axis 1 degenerate
  constexpr bool D2 = (DIM == 1);  // storage axis 2 degenerate
  __shared__ double red[kBlock / kWave];
  if (st != nullptr && st->done) return;  // uniform over the grid (a converged solve's queued launches)
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = threadIdx.x >> 6;
  int seg, j, kp;
  if (wmode == 0) {
    const int n1b = (g.n1 + 3) >> 2;
    const int b = blockIdx.x;
    seg = b % nseg;
    const int t = b / nseg;
    j = (t % n1b) * 4 + wave;
    kp = t / n1b;
  } else {
    const int gw = blockIdx.x * 4 + wave;
    seg = gw % nseg;
    const int row = gw / nseg;
    j = row % g.n1;
    kp = row / g.n1;
  }
  const int k = kfirst + kp;
  const bool row_ok = (j < g.n1) && (kp < nplanes);
  const int i = seg * kSeg - 1 + lane;
  const bool col_ok = row_ok && (i >= 0) && (i < g.n0);
  const int n0 = g.n0, n1 = g.n1, n2 = g.n2;
  const int64_t plane = (int64_t)n0 * n1;

  double bcoef = 0.0;
  bool first = false;
  // FUSEP: p ping-pongs between two buffers (in1 = buffer A, pout = buffer B) so
  // that p_old is never overwritten while neighbouring waves still read it.
  // Iteration `it` writes buffer (it & 1 ? B : A) and reads the other.
  const double* pold = in1;
  if (FUSEP) {
    const int it = st->it;
    first = (it == 0);
    bcoef = first ? 0.0 : st->beta / st->betaold;
    if (it & 1) {
      pold = in1;
    } else {
      pold = pout;
      pout = const_cast<double*>(in1);
    }
  }

  // ---- gather the 3x3 (j,k) column neighbourhood at x = i -------------------
  double X[3][3];   // stiffness input (T for RES, p for JAC)
  double Mm[3][3];  // mass input (T - Tp - dt f for RES)
#pragma unroll
  for (int b = 0; b < 3; ++b) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int jj = j + b - 1, kk = k + c - 1;
      const bool ok = col_ok && (D1 ? b == 1 : (jj >= 0 && jj < n1)) && (D2 ? c == 1 : (kk >= 0 && kk < n2));
      const int64_t idx = (int64_t)i + (int64_t)n0 * jj + plane * kk;
      double v = 0.0, v2 = 0.0;
      if (ok) {
        v = in0[idx];
        if (MODE == MODE_RES) v2 = in1[idx];
        if (FUSEP) v = first ? v : v + bcoef * pold[idx];
      }
      X[b][c] = v;
      if (MODE == MODE_RES) Mm[b][c] = v - v2 - g.dt_f;
    }
  }
  const double* cy = g.coef[1] + (int64_t)(j < n1 ? j : 0) * C_NCOEF;
  const double* cz = g.coef[2] + (int64_t)(k < n2 ? k : 0) * C_NCOEF;
  const double My[3] = {cy[C_MLO], cy[C_MDI], cy[C_MUP]};
  const double Ky[3] = {cy[C_KLO], cy[C_KDI], cy[C_KUP]};
  const double Mz[3] = {cz[C_MLO], cz[C_MDI], cz[C_MUP]};
  const double Kz[3] = {cz[C_KLO], cz[C_KDI], cz[C_KUP]};
  const double da = g.dt_alpha;

  // ---- fold y and z (sum factorisation) ---------------------------------------
  double S1 = 0.0, S2 = 0.0;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    double us = 0.0, vs = 0.0, um = 0.0;
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      us += My[b] * X[b][c];
      vs += Ky[b] * X[b][c];
      if (MODE == MODE_RES) um += My[b] * Mm[b][c];
    }
    if (MODE != MODE_RES) um = us;
    S1 += Mz[c] * (um + da * vs) + da * Kz[c] * us;
    S2 += Mz[c] * us;
  }
  S2 *= da;

  // ---- x direction via adjacent lanes ------------------------------------------
  const double S1m = shr1(S1), S1p = shl1(S1), S2m = shr1(S2), S2p = shl1(S2);
  const double* cx = g.coef[0] + (int64_t)(col_ok ? i : 0) * C_NCOEF;
  double y = 0.0;
  if (col_ok) {
    y = cx[C_MLO] * S1m + cx[C_MDI] * S1 + cx[C_MUP] * S1p + cx[C_KLO] * S2m + cx[C_KDI] * S2 +
        cx[C_KUP] * S2p;
  }

  // ---- Robin facets ---------------------------------------------------------------
  // faces normal to storage axis 2 (wave-uniform)
  if (!D2 && row_ok && ((k == 0 && g.bnd[2][0]) || (k == n2 - 1 && g.bnd[2][1]))) {
    double Tp_[3][3], Pp_[3][3];
#pragma unroll
    for (int v = 0; v < 3; ++v) {  // tangential axis 2 of the face = storage axis 1
      double pc = X[v][1], tc;
      if (MODE == MODE_RES) {
        tc = pc;
      } else {
        const int jj = j + v - 1;
        const bool ok = col_ok && (D1 ? v == 1 : (jj >= 0 && jj < n1));
        tc = ok ? T[(int64_t)i + (int64_t)n0 * jj + plane * k] : 0.0;
      }
      Tp_[0][v] = shr1(tc); Tp_[1][v] = tc; Tp_[2][v] = shl1(tc);
      Pp_[0][v] = shr1(pc); Pp_[1][v] = pc; Pp_[2][v] = shl1(pc);
    }
    if (col_ok) {
      y += facet_sum<MODE, false, false, D1>(g, cx[C_HLO], cx[C_HHI], cy[C_HLO], cy[C_HHI], Tp_, Pp_);
    }
  }
  // faces normal to storage axis 1 (wave-uniform)
  if (!D1 && row_ok && ((j == 0 && g.bnd[1][0]) || (j == n1 - 1 && g.bnd[1][1]))) {
    double Tp_[3][3], Pp_[3][3];
#pragma unroll
    for (int v = 0; v < 3; ++v) {  // tangential axes (0, 2)
      double pc = X[1][v], tc;
      if (MODE == MODE_RES) {
        tc = pc;
      } else {
        const int kk = k + v - 1;
        const bool ok = col_ok && (D2 ? v == 1 : (kk >= 0 && kk < n2));
        tc = ok ? T[(int64_t)i + (int64_t)n0 * j + plane * kk] : 0.0;
      }
      Tp_[0][v] = shr1(tc); Tp_[1][v] = tc; Tp_[2][v] = shl1(tc);
      Pp_[0][v] = shr1(pc); Pp_[1][v] = pc; Pp_[2][v] = shl1(pc);
    }
    if (col_ok) {
      y += facet_sum<MODE, false, false, D2>(g, cx[C_HLO], cx[C_HHI], cz[C_HLO], cz[C_HHI], Tp_, Pp_);
    }
  }
  // faces normal to storage axis 0 (lane-divergent: i == 0 or i == n0-1)
  if (col_ok && ((i == 0 && g.bnd[0][0]) || (i == n0 - 1 && g.bnd[0][1]))) {
    double Tp_[3][3];
    if (MODE == MODE_RES) {
#pragma unroll
      for (int u = 0; u < 3; ++u)
#pragma unroll
        for (int v = 0; v < 3; ++v) Tp_[u][v] = X[u][v];
    } else {
#pragma unroll
      for (int u = 0; u < 3; ++u) {
#pragma unroll
        for (int v = 0; v < 3; ++v) {
          const int jj = j + u - 1, kk = k + v - 1;
          const bool ok = (D1 ? u == 1 : (jj >= 0 && jj < n1)) && (D2 ? v == 1 : (kk >= 0 && kk < n2));
          Tp_[u][v] = ok ? T[(int64_t)i + (int64_t)n0 * jj + plane * kk] : 0.0;
        }
      }
    }
    y += facet_sum<MODE, false, D1, D2>(g, cy[C_HLO], cy[C_HHI], cz[C_HLO], cz[C_HHI], Tp_, X);
  }

  // ---- outputs --------------------------------------------------------------------
  const bool owned = (k >= g.k_begin) && (k < g.k_end);   // records
  const bool inwin = (k >= g.w_begin) && (k < g.w_end);   // writes (CgGrid: write window)
  const bool writer = col_ok && lane >= 1 && lane <= kSeg;
  const int64_t me = (int64_t)i + (int64_t)n0 * j + plane * k;
  if (writer) {
    if (FUSEP) pout[me] = X[1][1];
    if (inwin) out[me] = y;
  }
  if (MODE == MODE_JAC && partials != nullptr) {
    double d = (writer && owned) ? X[1][1] * y : 0.0;
    d = wave_sum(d);
    if (lane == 0) red[wave] = d;
    __syncthreads();
    if (threadIdx.x == 0) store_partial(&partials[blockIdx.x], (red[0] + red[1]) + (red[2] + red[3]));
  }
}


// ---------------------------------------------------------------------------
// diag(J): pointwise, facet terms with directly loaded patches.
// ---------------------------------------------------------------------------
// diag(J) at local node n; FACETS = false leaves out the Robin facet terms
template <int DIM, bool FACETS>
__device__ __forceinline__ double diag_value(const CgGrid& g, const double* __restrict__ T, int64_t n) {
  constexpr bool D1 = (DIM <= 2);
  constexpr bool D2 = (DIM == 1);
  const int64_t plane = (int64_t)g.n0 * g.n1;
  int i, j, k;
  decode_node(n, g, i, j, k);
  const double* cx = g.coef[0] + (int64_t)i * C_NCOEF;
  const double* cy = g.coef[1] + (int64_t)j * C_NCOEF;
  const double* cz = g.coef[2] + (int64_t)k * C_NCOEF;
  double d = cx[C_MDI] * cy[C_MDI] * cz[C_MDI] +
             g.dt_alpha * (cx[C_KDI] * cy[C_MDI] * cz[C_MDI] + cx[C_MDI] * cy[C_KDI] * cz[C_MDI] +
                           cx[C_MDI] * cy[C_MDI] * cz[C_KDI]);
  if (!FACETS) return d;
  auto load_patch = [&](int64_t stride_a, int64_t stride_b, bool dega, bool degb, int ia, int na, int ib, int nb,
                        double (&P)[3][3]) {
#pragma unroll
    for (int u = 0; u < 3; ++u)
#pragma unroll
      for (int v = 0; v < 3; ++v) {
        const int aa = ia + u - 1, bb = ib + v - 1;
        const bool ok = (dega ? u == 1 : (aa >= 0 && aa < na)) && (degb ? v == 1 : (bb >= 0 && bb < nb));
        P[u][v] = ok ? T[n + (int64_t)(u - 1) * stride_a + (int64_t)(v - 1) * stride_b] : 0.0;
      }
  };
  double P[3][3];
  if ((i == 0 && g.bnd[0][0]) || (i == g.n0 - 1 && g.bnd[0][1])) {
    load_patch(g.n0, plane, D1, D2, j, g.n1, k, g.n2, P);
    d += facet_sum<MODE_JAC, true, D1, D2>(g, cy[C_HLO], cy[C_HHI], cz[C_HLO], cz[C_HHI], P, P);
  }
  if (!D1 && ((j == 0 && g.bnd[1][0]) || (j == g.n1 - 1 && g.bnd[1][1]))) {
    load_patch(1, plane, false, D2, i, g.n0, k, g.n2, P);
    d += facet_sum<MODE_JAC, true, false, D2>(g, cx[C_HLO], cx[C_HHI], cz[C_HLO], cz[C_HHI], P, P);
  }
  if (!D2 && ((k == 0 && g.bnd[2][0]) || (k == g.n2 - 1 && g.bnd[2][1]))) {
    load_patch(1, g.n0, false, D1, i, g.n0, j, g.n1, P);
    d += facet_sum<MODE_JAC, true, false, D1>(g, cx[C_HLO], cx[C_HHI], cy[C_HLO], cy[C_HHI], P, P);
  }
  return d;
}

// all owned nodes; FACETS = false (3D marching path): the boundary nodes are
// rewritten by k_cg_diag_bnd, so no wave runs the facet sum for its one or two
// boundary lanes (every x-row has two)
template <int DIM, bool FACETS>
__global__ __launch_bounds__(kBlock) void k_cg_diag(CgGrid g, const double* __restrict__ T,
                                                    double* __restrict__ out, int invert) {
  const int64_t plane = (int64_t)g.n0 * g.n1;
  const int64_t nown = plane * (g.w_end - g.w_begin);  // the write window
  const int64_t base = plane * g.w_begin;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < nown;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t n = base + t;
    const double d = diag_value<DIM, FACETS>(g, T, n);
    out[n] = invert ? 1.0 / d : d;
  }
}

// the owned physical-boundary nodes (g.bnodes), facet terms included
__global__ __launch_bounds__(kBlock) void k_cg_diag_bnd(CgGrid g, const double* __restrict__ T,
                                                        double* __restrict__ out, int invert) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < g.n_bnodes;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t n = g.bnodes[t];
    const double d = diag_value<3, true>(g, T, n);
    out[n] = invert ? 1.0 / d : d;
  }
}


// ---------------------------------------------------------------------------
// 2.5D marching kernel (3D grids): the production matvec / residual.
//
// A workgroup = kRows wavefronts = kRows consecutive "rows" (along storage axis
// `raxis`) of one 64-wide x segment; it marches along the other axis (the
// "plane" axis) through a chunk of planes.  Per plane every lane loads ONE
// value of its own row (waves 0 / kRows-1 also load the two halo rows) into a
// double-buffered LDS slab, reads its j-1 / j / j+1 neighbours back, folds the
// row direction immediately (us = My.X, vs = Ky.X) and keeps (us, vs) of three
// consecutive planes in registers (sliding window).  The x direction is taken
// from the adjacent lanes with DPP.  HBM traffic ~ (kRows+2)/kRows x 8 B per
// input array per node; L2 and LDS carry the rest; one barrier per plane.
// Robin facets (<5% of nodes) gather their 3x3 patches directly.
// ---------------------------------------------------------------------------
constexpr int kRows = 8;       // rows (wavefronts) per marching workgroup
constexpr int kFaceChunk = 16;  // max planes per marching chunk (LDS coefficient stage)

template <int MODE, bool FUSEP>
__device__ double facet_direct(const CgGrid& g, int i, int j, int k, int ax, const double* __restrict__ T,
                               const double* __restrict__ in0, const double* pold, double bcoef, bool first) {
  const int t1 = (ax == 0) ? 1 : 0, t2 = (ax == 2) ? 1 : 2;
  const int c[3] = {i, j, k};
  const int n[3] = {g.n0, g.n1, g.n2};
  const int64_t st[3] = {1, g.n0, (int64_t)g.n0 * g.n1};
  const int64_t me = (int64_t)i + st[1] * j + st[2] * k;
  double Tp[3][3], Pp[3][3];
#pragma unroll
  for (int u = 0; u < 3; ++u)
#pragma unroll
    for (int v = 0; v < 3; ++v) {
      const int a = c[t1] + u - 1, b = c[t2] + v - 1;
      const bool ok = a >= 0 && a < n[t1] && b >= 0 && b < n[t2];
      const int64_t off = me + (int64_t)(u - 1) * st[t1] + (int64_t)(v - 1) * st[t2];
      if (MODE == MODE_RES) {
        Tp[u][v] = ok ? in0[off] : 0.0;
        Pp[u][v] = 0.0;
      } else {
        Tp[u][v] = ok ? T[off] : 0.0;
        double pv = ok ? in0[off] : 0.0;
        if (FUSEP && ok && !first) pv = pv + bcoef * pold[off];
        Pp[u][v] = pv;
      }
    }
  const double* c1 = g.coef[t1] + (int64_t)c[t1] * C_NCOEF;
  const double* c2 = g.coef[t2] + (int64_t)c[t2] * C_NCOEF;
  return facet_sum<MODE, false, false, false>(g, c1[C_HLO], c1[C_HHI], c2[C_HLO], c2[C_HHI], Tp, Pp);
}

// ---------------------------------------------------------------------------
// Robin facet Jacobian terms of the physical boundary faces,
//   fface[f][c_t1 + n_t1 c_t2] = dt sum_facets int g'(T_h) phi_I p_h ds
// (3x3 Gauss per facet, as facet_sum), evaluated matrix-free from the 3x3
// in-face patches of T and p, one thread per face node.  Nodes on two or
// three faces (edges, corners) get one term per face.
// ---------------------------------------------------------------------------
struct FaceOff {
  int off[7];  // workgroup ranges per face f (in marching-workgroup units), off[6] = total
};

// face tiles: kSeg nodes along t1 (one wavefront, two halo lanes) x (R - 1)
// node rows along t2 (R wavefronts: one facet row each, see face_block).  The
// faces normal to the march axis `qaxis` are integrated inside the marching
// tiles instead (k_cg_march) and get no face tiles.
FaceOff face_offsets(const CgGrid& g, int R, int qaxis) {
  FaceOff fo{};
  int acc = 0;
  const int rows = R - 1;
  for (int f = 0; f < 6; ++f) {
    fo.off[f] = acc;
    if (g.fface[f] && (f >> 1) != qaxis) acc += ((g.fn1[f] + kSeg - 1) / kSeg) * ((g.fn2[f] + rows - 1) / rows);
  }
  fo.off[6] = acc;
  return fo;
}

// Robin facet Jacobian of ONE facet (c1, c1+1) x (row, row+1) of a boundary
// face: the corner contributions dt int_f g'(T_h) phi_X p_h ds for X = a (c1,
// row), b (c1+1, row), c (c1, row+1), d (c1+1, row+1), 3x3 Gauss points (exact
// for the degree-5 per direction integrand).  Ta/Tc, Pa/Pc: T and p at the
// lane's node of the lower / upper row; the c1+1 values come from the next lane
// (DPP), so every lane of the wave must call this (uniform control flow).
__device__ __forceinline__ void facet_corners(const CgGrid& g, bool ok, double h1, double h2, double Ta,
                                              double Tc, double Pa, double Pc, double& ya, double& yb,
                                              double& yc, double& yd) {
  const double Tb = shl1(Ta), Td = shl1(Tc), Pb = shl1(Pa), Pd = shl1(Pc);
  ya = yb = yc = yd = 0.0;
  if (ok) {
#pragma unroll
    for (int q1 = 0; q1 < 3; ++q1) {
#pragma unroll
      for (int q2 = 0; q2 < 3; ++q2) {
        const double sx = kGX[q1], tx = kGX[q2];
        const double fa = (1.0 - sx) * (1.0 - tx), fb = sx * (1.0 - tx), fc = (1.0 - sx) * tx, fd = sx * tx;
        const double Th = fa * Ta + fb * Tb + fc * Tc + fd * Td;
        const double Ph = fa * Pa + fb * Pb + fc * Pc + fd * Pd;
        const double G = (kGW[q1] * kGW[q2]) * dg_rad_conv(g, Th) * Ph;
        ya += G * fa;
        yb += G * fb;
        yc += G * fc;
        yd += G * fd;
      }
    }
    const double sc = g.dt * (h1 * h2);
    ya *= sc; yb *= sc; yc *= sc; yd *= sc;
  }
}

// One face workgroup of the marching launch (Jacobian mode): the Robin facet
// Jacobian terms dt * int_f g'(T_h) phi_I p_h ds of a tile of face nodes,
// evaluated per FACET: lane = facet (c1, c1+1) x (f, f+1) of wave w's facet
// row f = r0 - 1 + w; its 9 Gauss points (3x3, exact for the degree-5 per
// direction integrand) give the four corner contributions at once (4x less
// arithmetic than integrating the up-to-4 facets of every node separately).
// A node sums the corners of its 4 facets: t1 neighbours by DPP, the facet
// row below through LDS.  T and p (p = z + beta/betaold p_old in the fused
// PCG, else p = x) of the R + 1 node rows r0-1 .. r0+R-1 are staged in LDS;
// waves 1..R-1 write node rows r0 .. r0+R-2 of fface and the workgroup's
// p.(facet terms) record, then the tile takes part in the reduction tail.
template <bool FUSEP, int R>
__device__ void face_block(const CgGrid& g, const double* __restrict__ T, const double* __restrict__ in0,
                           const double* pA, const double* pB, double beta_ratio,
                           double* __restrict__ partials, const RedTail& rt, int nrec, int fb,
                           const FaceOff& fo, double* sm, double* redf, int it_host) {
  // LDS carved from the kernel's shared buffer (the marching tiles use it for
  // their own face planes): T and p of R + 1 node rows, and the upper-corner
  // contributions (c: c1, d: c1 + 1) of each facet row
  double (*sT)[kWave] = reinterpret_cast<double (*)[kWave]>(sm);
  double (*sP)[kWave] = reinterpret_cast<double (*)[kWave]>(sm + (R + 1) * kWave);
  double (*sCD)[R][kWave] = reinterpret_cast<double (*)[R][kWave]>(sm + 2 * (R + 1) * kWave);
  int f = 0;
  while (f < 5 && fb >= fo.off[f + 1]) ++f;
  const int a = f >> 1, side = f & 1;
  const int t1 = (a == 0) ? 1 : 0, t2 = (a == 2) ? 1 : 2;
  const int n[3] = {g.n0, g.n1, g.n2};
  const int sst[3] = {1, g.n0, g.n0 * g.n1};
  const int n1 = n[t1], n2 = n[t2];
  const int nseg1 = (n1 + kSeg - 1) / kSeg;
  const int tile = fb - fo.off[f];
  const int seg = tile % nseg1, tb = tile / nseg1;
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c1 = seg * kSeg - 1 + lane;
  const int r0 = tb * (R - 1);
  const bool ok1 = c1 >= 0 && c1 < n1;
  double bcoef = 0.0;
  bool first = true;
  const double* pold = pA;
  if (FUSEP) {  // iteration parity from the host (no dependent load before the staging loads)
    first = (it_host == 0);
    bcoef = first ? 0.0 : beta_ratio;
    pold = (it_host & 1) ? pA : pB;
  }
  auto node_of = [&](int cc1, int cc2) {
    int c[3];
    c[t1] = cc1;
    c[t2] = cc2;
    c[a] = side ? n[a] - 1 : 0;
    return c[0] + sst[1] * c[1] + sst[2] * c[2];
  };
  // staging in two halves: every row's loads first (wave R - 1 stages two
  // rows), then the LDS stores -- storing the first row before loading the
  // second made that wave, and through the barrier the workgroup, wait for two
  // memory round trips
  struct Stg {
    double tt, zz, oo;
    bool ok;
  };
  auto stage_ld = [&](int cc2) -> Stg {
    const bool ok = ok1 && cc2 >= 0 && cc2 < n2;
    const int o = ok ? node_of(c1, cc2) : 0;
    return Stg{T[o], in0[o], FUSEP ? pold[o] : 0.0, ok};
  };
  auto stage_st = [&](int row, const Stg& v) {
    sT[row][lane] = v.ok ? v.tt : 0.0;
    sP[row][lane] = v.ok ? ((FUSEP && !first) ? v.zz + bcoef * v.oo : v.zz) : 0.0;
  };
  // facet (c1, c1 + 1) x (fr, fr + 1), corners a = (c1, fr), b = (c1+1, fr),
  // c = (c1, fr+1), d = (c1+1, fr+1); its cell lengths load with the staging
  const int fr = r0 - 1 + wave;
  const bool facet_ok = c1 >= 0 && c1 < n1 - 1 && fr >= 0 && fr < n2 - 1;
  const double h1 = g.coef[t1][(int64_t)(facet_ok ? c1 : 0) * C_NCOEF + C_HHI];
  const double h2 = g.coef[t2][(int64_t)(facet_ok ? fr : 0) * C_NCOEF + C_HHI];
  const Stg sa = stage_ld(r0 - 1 + wave);
  Stg sb{0.0, 0.0, 0.0, false};
  if (wave == R - 1) sb = stage_ld(r0 + R - 1);  // wave-uniform
  stage_st(wave, sa);
  if (wave == R - 1) stage_st(R, sb);
  __syncthreads();
  const double Pa = sP[wave][lane];
  double ya, yb, yc, yd;
  facet_corners(g, facet_ok, h1, h2, sT[wave][lane], sT[wave + 1][lane], Pa, sP[wave + 1][lane], ya, yb, yc, yd);
  sCD[0][wave][lane] = yc;
  sCD[1][wave][lane] = yd;
  const double ybl = shr1(yb);  // facet (c1 - 1) contributes its b corner to node c1
  __syncthreads();
  double dot = 0.0;
  const int c2 = r0 - 1 + wave;  // node row of wave w (w >= 1)
  const bool wr = wave >= 1 && ok1 && lane >= 1 && lane <= kSeg && c2 < n2;
  if (wr) {
    // facets below (row c2 - 1): corners c (same c1) and d (from c1 - 1)
    const double acc = (ya + ybl) + (sCD[0][wave - 1][lane] + sCD[1][wave - 1][lane - 1]);
    int c[3];
    c[t1] = c1;
    c[t2] = c2;
    c[a] = side ? n[a] - 1 : 0;
    const bool owned = c[2] >= g.k_begin && c[2] < g.k_end;
    g.fface[f][c1 + n1 * c2] = (c[2] >= g.w_begin && c[2] < g.w_end) ? acc : 0.0;
    dot = owned ? Pa * acc : 0.0;
  }
  if (partials != nullptr) {
    dot = wave_sum(dot);
    if (lane == 0) redf[wave] = dot;
    __syncthreads();
    if (threadIdx.x == 0) {
      double s2 = 0.0;
#pragma unroll
      for (int w = 0; w < R; ++w) s2 += redf[w];
      store_partial(&partials[blockIdx.x], s2);
    }
    fused_reduce_tail<1>(rt, nrec);
  }
}

// out[n] += sum of the facet terms of the owned boundary node n (every face
// it lies on), for the non-fused J(T) x
// Only the nodes of the face-workgroup faces are visited (normal to storage
// axis 0 and to the row axis raxis; the faces along the march axis are
// integrated inside the tiles): x faces for every owned (j, k), row-axis faces
// for i in [1, n0 - 2] (edge nodes are x-face nodes, every face of a node is
// summed there).  At C4 that is 82 K nodes instead of the 403 K boundary nodes
// (7.0 -> ~3 us per complete J x).
__global__ __launch_bounds__(kBlock) void k_cg_addfaces(CgGrid g, double* __restrict__ out, int raxis,
                                                        const PcgState* __restrict__ st) {
  if (st != nullptr && st->done) return;  // queued behind a converged solve (multigrid V-cycle)
  const int n[3] = {g.n0, g.n1, g.n2};
  const int kb = g.w_begin, nk = g.w_end - g.w_begin;  // the write window
  const int sx = n[0] > 1 ? 2 : 1;
  const int64_t nA = (int64_t)sx * n[1] * nk;
  // row-axis faces: raxis 1 -> j in {0, n1 - 1} x owned k; raxis 2 -> the owned ones of k in {0, n2 - 1} x j
  const int nin = n[0] - 2 > 0 ? n[0] - 2 : 0;
  const int nfree = (raxis == 1) ? nk : n[1];
  const int64_t nB = 2 * (int64_t)nin * nfree;
  // the face terms and the node's output through buffer loads issued together
  // (out-of-range offsets where a face does not apply): loaded under the face
  // tests, each was waited for at once and the output load after them
  const double* fb = nullptr;
#pragma unroll
  for (int f = 0; f < 6; ++f)
    if (fb == nullptr && g.fface[f] != nullptr) fb = g.fface[f] - g.ffoff[f];
  const buf_t rsF = mk_rsrc(fb, fb ? (uint32_t)(g.ffsize * 8) : 0u);
  const uint32_t obytes = (uint32_t)n[0] * (uint32_t)n[1] * (uint32_t)n[2] * 8u;
  const buf_t rsO = mk_rsrc(out, obytes);
  const int fr_lo = (raxis == 1) ? 2 : 4;
  for (int64_t e = blockIdx.x * (int64_t)kBlock + threadIdx.x; e < nA + nB; e += (int64_t)gridDim.x * kBlock) {
    int c[3];
    if (e < nA) {
      const int64_t pl = (int64_t)n[1] * nk;
      const int side = (int)(e / pl);
      const int64_t r = e - side * pl;
      c[0] = side ? n[0] - 1 : 0;
      c[1] = (int)(r % n[1]);
      c[2] = kb + (int)(r / n[1]);
    } else {
      const int64_t u = e - nA, pl = (int64_t)nin * nfree;
      const int side = (int)(u / pl);
      const int64_t r = u - side * pl;
      c[0] = 1 + (int)(r % nin);
      const int o = (int)(r / nin);
      if (raxis == 1) {
        c[1] = side ? n[1] - 1 : 0;
        c[2] = kb + o;
      } else {
        c[1] = o;
        c[2] = side ? n[2] - 1 : 0;
        if (c[2] < kb || c[2] >= g.w_end) continue;  // that plane is not in the write window
      }
    }
    // x faces (index c1 + n1 c2), then the row-axis faces (index c0 + n0 c_t2):
    // the order of the face loop this replaced, so the sums are bitwise the same
    const bool x0 = g.fface[0] && c[0] == 0, x1 = g.fface[1] && c[0] == n[0] - 1;
    const bool r0 = g.fface[fr_lo] && c[raxis] == 0, r1 = g.fface[fr_lo + 1] && c[raxis] == n[raxis] - 1;
    const int rt2 = (raxis == 1) ? c[2] : c[1];
    const int64_t ex = (x0 ? g.ffoff[0] : g.ffoff[1]) + c[1] + (int64_t)n[1] * c[2];
    const int64_t er = (r0 ? g.ffoff[fr_lo] : g.ffoff[fr_lo + 1]) + c[0] + (int64_t)n[0] * rt2;
    const uint32_t oq = (uint32_t)(c[0] + (int64_t)n[0] * (c[1] + (int64_t)n[1] * c[2])) * 8u;
    const double fx = bload(rsF, (x0 || x1) ? (uint32_t)ex * 8u : kBadOff);
    const double fr = bload(rsF, (r0 || r1) ? (uint32_t)er * 8u : kBadOff);
    const double old = bload(rsO, oq);
    const double add = fx + fr;
    if (add != 0.0) bstore(rsO, oq, old + add);
  }
}

// Tile of marching workgroup bid.  Each XCD (bid & 7) takes a contiguous
// share of the tile sequence (as xcd_remap), and that share BEGINS with its
// part of the face-chunk tiles: the first and the last chunk along the march
// axis integrate the Robin facets of the faces normal to it in their
// prologue, so those tiles run longer.  In plain chunk order they sat on the
// XCDs holding the first and last chunks (C4: 4 chunks, XCDs 0-1 and 6-7) and
// ran last there; here every XCD gets the same number of them, first (C4:
// fused matvec 74.1 -> 72.0 us, J x 41.8 -> 40.5 us, flushed J x 52.5 ->
// 50.9 us, interleaved A/B on one box).  Face tiles: seg fastest, then row
// block, then face chunk; the others: seg, row block, chunk 1 .. nch - 2 --
// XCD x works on the same band of row blocks in both parts.
__device__ __forceinline__ void march_tile(int bid, int nmarch, int nseg, int nrbk, int nch, int& seg, int& rb,
                                           int& chunk) {
  const int x = bid & 7, p = bid >> 3;
  const int q = nmarch >> 3, r = nmarch & 7;
  const int start = x * q + min(x, r);
  const int per_chunk = nseg * nrbk;
  const int nF = (nch > 1 ? 2 : 1) * per_chunk;
  const int fq = nF >> 3, fr = nF & 7;
  const int fsize = fq + (x < fr ? 1 : 0), fstart = x * fq + min(x, fr);
  int t, c;
  if (p < fsize) {
    t = fstart + p;
    c = t / per_chunk;
    chunk = c ? nch - 1 : 0;
  } else {
    t = (start - fstart) + (p - fsize);
    c = t / per_chunk;
    chunk = 1 + c;
  }
  t -= c * per_chunk;
  seg = t % nseg;
  rb = t / nseg;
}

// WPE: minimum waves per SIMD the register allocation must allow (8: <= 64
// VGPRs, four 8-wave tiles per CU, at the price of a few spills)
// PF: prefetch depth (planes whose loads are in flight while one is computed)
// POST (MODE_JAC, !FUSEP): the multigrid's level-0 post-smoothing in the
// epilogue -- out = z = x + omega dinv (r - J x) instead of J x, with r and dinv
// of the output plane in the prefetch ring, and (z.z, z.r) per tile as records
// 2 tile, 2 tile + 1; the facet terms of the face workgroups (faces along the
// march) are applied afterwards by k_mg_post_faces, which also runs the tail.
template <int MODE, bool FUSEP, int R, int WPE, int PF, bool POST = false>
__global__ __launch_bounds__(R * kWave) __attribute__((amdgpu_waves_per_eu(WPE))) void k_cg_march(CgGrid g, const double* __restrict__ T,
                                                        const double* __restrict__ in0, const double* in1,
                                                        double* __restrict__ out, double* pout,
                                                        const PcgState* __restrict__ st,
                                                        double* __restrict__ partials, int nseg, int raxis,
                                                        int qchunk, RedTail rt, int nrec, int nmarch,
                                                        FaceOff fo, int it_host, PostArgs pa) {
  static_assert(!POST || (MODE == MODE_JAC && !FUSEP), "POST: plain Jacobian march only");
  stamp_start(rt);
  constexpr int NA = (MODE == MODE_RES) ? 2 : 1;  // LDS arrays: stiffness input (+ mass input)
  __shared__ double lds[NA][2][R + 2][kWave];  // double-buffered plane slab (one barrier per plane)
  __shared__ double red[R];
  // face LDS: face workgroups (face_block) or the marching tiles' own face
  // planes -- [2 faces][T, p][R + 2 rows] slabs + corner exchange [2 faces][c, d][R rows]
  constexpr int kFaceLds = (MODE == MODE_JAC) ? (8 * R + 8) * kWave : 1;
  __shared__ double fsm[kFaceLds];
  // Jacobian mode: workgroups past the marching tiles evaluate the Robin facet
  // terms of the boundary faces (face_block) -- independent work that fills
  // the tail of the march; the terms go to g.fface and are added to w by the
  // consumer (PCG update / k_cg_addfaces), their p.w share joins the partials
  // (placed before the tiles or interleaved with them: measured no better)
  const int bid = (int)blockIdx.x;
  const int fidx = (MODE == MODE_JAC && bid >= nmarch) ? bid - nmarch : -1;
  // lagged logic (multi-rank fused matvec): the state after the previous
  // all-reduce is formed here and committed by the tail (lagged_state)
  const bool lagged = FUSEP && rt.lag != nullptr;
  if (lagged && bid == 0 && threadIdx.x == 0) {
    // a lagged state that ends the solve is committed here, by workgroup 0
    // before it has anything in flight (every workgroup then exits; formed
    // here rather than at the exit test below, where the full logic would
    // raise the kernel's register count); otherwise the tail commits it
    // (written through rt.st: st itself stays read-only, so the compiler keeps
    // its reads scalar and ahead of nothing)
    const PcgState s = lagged_state(st, rt.lag, rt.lag_kind);
    if (s.done) *rt.st = s;
  }
  if (fidx >= 0) {
    double ratio = 0.0;
    if (lagged) {
      int ldone;
      double lbeta;
      lag_update_lean(st, rt.lag, ldone, lbeta);
      if (ldone) return;
      ratio = lbeta / st->betaold;
    } else if (st != nullptr) {
      if (st->done) return;
      if (FUSEP) ratio = st->beta / st->betaold;
    }
    face_block<FUSEP, R>(g, T, in0, in1, pout, ratio, POST ? nullptr : partials, POST ? RedTail{} : rt, nrec, fidx, fo,
                         fsm, red, it_host);
    return;
  }
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int n0 = g.n0;
  const int nR = (raxis == 1) ? g.n1 : g.n2;
  const int nQ = (raxis == 1) ? g.n2 : g.n1;
  const int64_t sR = (raxis == 1) ? (int64_t)n0 : (int64_t)n0 * g.n1;
  const int64_t sQ = (raxis == 1) ? (int64_t)n0 * g.n1 : (int64_t)n0;
  // tile order (march_tile): x segment fastest, then row block, then chunk;
  // each XCD takes a contiguous run of tiles, i.e. whole x-rows of a band of row
  // blocks in one chunk -- the concurrent tiles of an XCD read long contiguous
  // runs and share their halo rows in L2 (measured at C4 against chunk-fastest:
  // step 11.22 / 11.34 -> 10.99 / 10.85 ms, flushed J x 53.5 -> 50.9-52.6 us;
  // segment, then chunk: 11.08 / 11.17 ms)
  const int nch = (nQ + qchunk - 1) / qchunk;
  const int nrbk = (nR + R - 1) / R;
  int seg, rb, chunk;
  march_tile(bid, nmarch, nseg, nrbk, nch, seg, rb, chunk);
  const int r0 = rb * R;
  const int r = r0 + wave;
  const bool row_ok = r < nR;
  const int q0 = chunk * qchunk;
  const int q1 = min(q0 + qchunk, nQ);
  const int i = seg * kSeg - 1 + lane;
  const bool col_ok = (i >= 0) && (i < n0);
  const bool writer = col_ok && lane >= 1 && lane <= kSeg;

  double bcoef = 0.0;
  bool first = false;
  const double* pold = in1;
  if (FUSEP) {  // iteration parity from the host: the prefetch does not wait for a load of st
    first = (it_host == 0);
    if (!(it_host & 1)) { pold = pout; pout = const_cast<double*>(in1); }
  }
  // the solver state (scalar loads, issued first; read after the block's
  // loads are all in flight)
  int st_done = 0;
  double st_beta = 0.0, st_betaold = 1.0;
  if (lagged) {  // the multi-rank solves lag logic_update (kind 3) into this launch
    lag_update_lean(st, rt.lag, st_done, st_beta);
    st_done = __builtin_amdgcn_readfirstlane(st_done);  // wave-uniform: keep them in SGPRs
    st_beta = uniform(st_beta);
    st_betaold = st->betaold;
  } else if (st != nullptr) {
    st_done = st->done;
    if (FUSEP) {
      st_beta = st->beta;
      st_betaold = st->betaold;
    }
  }
  // ownership along storage axis 2 (partition axis): outputs on the write
  // window, the records (p.w, z.z, z.r) over the owned planes
  const int kb = g.k_begin, ke = g.k_end, wb = g.w_begin, we = g.w_end;
  const bool row_owned = (raxis == 2) ? (r >= kb && r < ke) : true;
  const bool row_inwin = (raxis == 2) ? (r >= wb && r < we) : true;
  // per-axis data of the row / march axes by selects, not by indexing the
  // kernel arguments with a runtime axis (each such index is a dependent
  // scalar load of the argument segment ahead of the first memory request)
  const double* coefR = (raxis == 1) ? g.coef[1] : g.coef[2];
  const double* coefQ = (raxis == 1) ? g.coef[2] : g.coef[1];
  const int bq_lo = (raxis == 1) ? g.bnd[2][0] : g.bnd[1][0];
  const int bq_hi = (raxis == 1) ? g.bnd[2][1] : g.bnd[1][1];

  // Robin facet terms of the faces normal to the march axis (Jacobian): the
  // tile's first / last chunk holds that face's plane.  They are integrated in
  // the tile's prologue -- T and p of the face plane's R + 2 rows staged in
  // LDS, one facet row per wave (wave 0 also the row below the tile), corner
  // exchange through LDS -- and added to that plane's output in the march.
  const bool fq0 = (MODE == MODE_JAC) && q0 == 0 && bq_lo;
  const bool fq1 = (MODE == MODE_JAC) && q1 == nQ && bq_hi;
  double (*sFq)[2][R + 2][kWave] = reinterpret_cast<double (*)[2][R + 2][kWave]>(fsm);  // [face][T, p]
  double (*sCD)[2][R][kWave] = reinterpret_cast<double (*)[2][R][kWave]>(fsm + 4 * (R + 2) * kWave);
  double yq0 = 0.0, yq1 = 0.0;
  const double da = g.dt_alpha;

  // raw loads of one (row, plane) value (+ second array); the combination
  // (p = z + b p_old, or T - Tp - dt f) happens one iteration later so the
  // loads of plane L+1 are in flight while plane L is processed.  Buffer
  // loads: a per-lane row offset (fixed for the march) plus a uniform plane
  // offset; anything outside the domain reads 0 (range check).
  const double* second = (MODE == MODE_RES) ? in1 : pold;
  constexpr bool TWO = (MODE == MODE_RES) || FUSEP;
  const uint32_t nbytes = (uint32_t)g.n0 * (uint32_t)g.n1 * (uint32_t)g.n2 * 8u;
  const buf_t rs0 = mk_rsrc(in0, nbytes);
  const buf_t rs1 = mk_rsrc(TWO ? second : in0, (FUSEP && first) ? 0u : nbytes);  // p_old unused at it 0
  const buf_t rso = mk_rsrc(out, nbytes);
  const buf_t rsp = mk_rsrc(FUSEP ? pout : out, FUSEP ? nbytes : 0u);
  const buf_t rsT = mk_rsrc(T, (fq0 || fq1) ? nbytes : 0u);
  const buf_t rsZ = mk_rsrc(in0, (fq0 || fq1) ? nbytes : 0u);
  const buf_t rsO = mk_rsrc(TWO ? second : in0, ((fq0 || fq1) && FUSEP && !first) ? nbytes : 0u);
  // halo rows are loaded by waves 0 and R-1; the other waves re-load their own
  // row (an L1 hit) so that every wave runs the same straight-line load stream
  const bool halo = (wave == 0) || (wave == R - 1);
  const int hrow = (wave == 0) ? r0 - 1 : (wave == R - 1 ? r0 + R : r);
  const int hslot = (wave == 0) ? 0 : R + 1;
  auto lane_off = [&](int rr) -> uint32_t {
    return (col_ok && rr >= 0 && rr < nR) ? (uint32_t)(i + sR * rr) * 8u : kBadOff;
  };
  // the halo row offset of the other waves is out of range: their halo loads
  // return 0 without a memory request, the instruction stream stays uniform
  const uint32_t vo_own = lane_off(r), vo_halo = halo ? lane_off(hrow) : kBadOff;
  const uint32_t vo_wr = writer ? vo_own : kBadOff;  // stores of the own row
  auto plane_off = [&](int L) -> uint32_t { return (L >= 0 && L < nQ) ? (uint32_t)(sQ * L) * 8u : kBadOff; };
  // (a streaming policy for these loads, bload_nt, measured no gain; a runtime
  // switch between the two costs a scalar branch per load in the march)
  auto fetch = [&](uint32_t vo, int L, double& a0, double& a1) {
    const uint32_t o = vo + plane_off(L);
    a0 = bload(rs0, o);
    a1 = TWO ? bload(rs1, o) : 0.0;
  };
  // POST: r and dinv of the own row at plane L - 1 (the output plane of step L).
  // D^-1 is loaded on the physical-boundary nodes only (their Robin facet
  // terms, rewritten every Newton iteration; Dirichlet zeros): everywhere else
  // step() forms 1 / diag(M + dt alpha K) from the staged axis coefficients
  // (8 B per node fewer; the other lanes' loads carry an out-of-range offset)
  const buf_t rsr = mk_rsrc(pa.r, POST ? nbytes : 0u);
  const buf_t rsd = mk_rsrc(pa.dinv, POST ? nbytes : 0u);
  const int bR_lo = (raxis == 1) ? g.bnd[1][0] : g.bnd[2][0], bR_hi = (raxis == 1) ? g.bnd[1][1] : g.bnd[2][1];
  const bool bnd_lr = (i == 0) || (i == n0 - 1) || (r == 0 && bR_lo) || (r == nR - 1 && bR_hi);  // x face, row face
  auto bnd_q = [&](int q) { return (q == 0 && bq_lo) || (q == nQ - 1 && bq_hi); };    // march-axis face
  auto fetch_post = [&](int L, double& a_r, double& a_d) {
    if (!POST) return;
    const uint32_t o = vo_wr + plane_off(L - 1);
    a_r = bload(rsr, o);
    a_d = bload(rsd, (bnd_lr || bnd_q(L - 1)) ? o : kBadOff);
  };

  auto combine = [&](uint32_t vo, int L, double a0, double a1, double& v, double& vm) {
    v = a0;
    vm = 0.0;
    if (MODE == MODE_RES) vm = (vo != kBadOff && L >= 0 && L < nQ) ? a0 - a1 - g.dt_f : 0.0;
    if (FUSEP) v = a0 + bcoef * a1;  // a1 = 0 and bcoef = 0 at the first iteration
  };
  // Block start: ONE memory round trip for everything the march needs before
  // its first plane -- the first two planes (prefetch), the coefficient
  // stages (march axis, x axis, the tile's rows) and the face planes of the
  // Robin facets -- issued back to back, prefetch first, all before the
  // solver state is tested.  (Round 4: the row coefficients used to be read
  // per wave ahead of the prefetch, and the stages only after the state test,
  // so a tile waited for three memory round trips before its first plane.)
  // prefetch ring: PF + 1 register sets rotate through a fully unrolled loop,
  // so PF planes of loads are in flight while a plane is combined, exchanged
  // and computed
  double ra0[PF + 1], ra1[PF + 1], rh0[PF + 1], rh1[PF + 1];
  double rr[PF + 1], rd[PF + 1];  // POST: r, dinv of the output plane
#pragma unroll
  for (int s = 0; s < PF; ++s) {
    fetch(vo_own, q0 - 1 + s, ra0[s], ra1[s]);
    fetch(vo_halo, q0 - 1 + s, rh0[s], rh1[s]);
    fetch_post(q0 - 1 + s, rr[s], rd[s]);
  }
  // march-axis coefficients of the chunk, pre-scaled per plane q into
  // (Mz0, Mz1, Mz2, da Kz0, da Kz1, da Kz2, da Mz0, da Mz1, da Mz2, 0): read
  // as 5 uniform 16-byte LDS loads per plane; x-axis coefficients of the
  // block's 64 columns as (Mlo, Klo), (Mdi, Kdi), (Mup, Kup), (Hhi, -) pairs
  // per lane: 3 conflict-free 16-byte LDS loads per plane; the coefficients
  // of the tile's rows r0 - 1 .. r0 + R - 1 (row slot + 1), read per wave
  // into SGPRs after the barrier
  __shared__ double2 cql[kFaceChunk + 2][5];
  __shared__ double2 cxl[4][kWave];
  __shared__ double crl[R + 1][C_NCOEF];
  const int nqs = q1 - q0 + 2;
  const bool st_q = (int)threadIdx.x < nqs * 6;
  const bool st_x = (int)threadIdx.x < 8 * kWave;
  const bool st_r = (int)threadIdx.x < (R + 1) * C_NCOEF;
  double cqv, cxv, crv;
  {
    const int e = threadIdx.x;
    const int qq = q0 - 1 + e / 6;
    const bool okq = st_q && qq >= 0 && qq < nQ;
    cqv = coefQ[okq ? (int64_t)qq * C_NCOEF + e % 6 : 0];
    const int ii = seg * kSeg - 1 + (e & (kWave - 1));
    const bool okx = st_x && ii >= 0 && ii < n0;
    const int k = e >> 6;  // slot: pair k >> 1, half k & 1
    const int cc = k == 0 ? C_MLO : k == 1 ? C_KLO : k == 2 ? C_MDI : k == 3 ? C_KDI : k == 4 ? C_MUP : k == 5 ? C_KUP : C_HHI;
    cxv = g.coef[0][okx ? (int64_t)ii * C_NCOEF + cc : 0];
    const int rrow = r0 - 1 + e / C_NCOEF;
    const bool okr = st_r && rrow >= 0 && rrow < nR;
    crv = coefR[okr ? (int64_t)rrow * C_NCOEF + e % C_NCOEF : 0];
    cqv = okq ? cqv : 0.0;
    cxv = (okx && k < 7) ? cxv : 0.0;
    crv = okr ? crv : 0.0;
  }
  // face planes: T, z (, p_old) of the own and halo rows
  double fT[2][2], fZ[2][2], fO[2][2];  // [face][own, halo]
  if (fq0 || fq1) {
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      const uint32_t po = plane_off(f == 0 ? (fq0 ? 0 : -1) : (fq1 ? nQ - 1 : -1));
      fT[f][0] = bload(rsT, vo_own + po); fT[f][1] = bload(rsT, vo_halo + po);
      fZ[f][0] = bload(rsZ, vo_own + po); fZ[f][1] = bload(rsZ, vo_halo + po);
      fO[f][0] = FUSEP ? bload(rsO, vo_own + po) : 0.0;
      fO[f][1] = FUSEP ? bload(rsO, vo_halo + po) : 0.0;
    }
  }
  // once the PCG has converged every launch of the batch exits here (a plain
  // J x inside a converged solve's queued V-cycle too)
  if (st_done) return;
  if (FUSEP) bcoef = first ? 0.0 : st_beta / st_betaold;
  if (st_q) {
    const int qs = threadIdx.x / 6, c = threadIdx.x % 6;
    double* row = reinterpret_cast<double*>(cql[qs]);
    if (c < 3) {
      row[c] = cqv;            // Mz
      row[6 + c] = da * cqv;   // da Mz
    } else {
      row[c] = da * cqv;       // da Kz
    }
    if (c == 0) row[9] = 0.0;
  }
  if (st_x) reinterpret_cast<double*>(cxl[(threadIdx.x >> 6) >> 1])[2 * (threadIdx.x & (kWave - 1)) + ((threadIdx.x >> 6) & 1)] = cxv;
  if (st_r) crl[threadIdx.x / C_NCOEF][threadIdx.x % C_NCOEF] = crv;
  if (fq0 || fq1) {
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      sFq[f][0][wave + 1][lane] = fT[f][0];
      sFq[f][1][wave + 1][lane] = FUSEP ? fZ[f][0] + bcoef * fO[f][0] : fZ[f][0];
      if (halo) {
        sFq[f][0][hslot][lane] = fT[f][1];
        sFq[f][1][hslot][lane] = FUSEP ? fZ[f][1] + bcoef * fO[f][1] : fZ[f][1];
      }
    }
  }
  __syncthreads();
  // row coefficients are wave-uniform: keep them in SGPRs (row slot wave + 1;
  // zeros past the last row, as before)
  const double* crw = crl[wave + 1];
  const double My0 = uniform(crw[C_MLO]), My1 = uniform(crw[C_MDI]), My2 = uniform(crw[C_MUP]);
  const double Ky0 = uniform(crw[C_KLO]), Ky1 = uniform(crw[C_KDI]), Ky2 = uniform(crw[C_KUP]);
  // facet-row cell lengths along the row axis (own facet row r; r0 - 1 for wave 0)
  const double hq_own = uniform(crw[C_HHI]);
  const double hq_low = uniform(crl[0][C_HHI]);
  if (fq0 || fq1) {  // facet row r (rows r, r + 1) of each face plane; wave 0 also row r0 - 1
    const bool cok = i >= 0 && i < n0 - 1;
    const double h1 = cxl[3][lane].x;
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      if (!(f == 0 ? fq0 : fq1)) continue;  // block-uniform: only the face planes this chunk holds
      double ya, yb, yc, yd;
      facet_corners(g, cok && r < nR - 1, h1, hq_own, sFq[f][0][wave + 1][lane], sFq[f][0][wave + 2][lane],
                    sFq[f][1][wave + 1][lane], sFq[f][1][wave + 2][lane], ya, yb, yc, yd);
      double yq = ya + shr1(yb);
      sCD[f][0][wave][lane] = yc;
      sCD[f][1][wave][lane] = yd;
      if (wave == 0) {
        facet_corners(g, cok && r0 >= 1 && r0 - 1 < nR - 1, h1, hq_low, sFq[f][0][0][lane], sFq[f][0][1][lane],
                      sFq[f][1][0][lane], sFq[f][1][1][lane], ya, yb, yc, yd);
        yq += yc + shr1(yd);
      }
      if (f == 0) yq0 = yq; else yq1 = yq;
    }
    __syncthreads();
    if (wave >= 1) {
      const int lm = lane >= 1 ? lane - 1 : 0;
      yq0 += sCD[0][0][wave - 1][lane] + sCD[0][1][wave - 1][lm];
      yq1 += sCD[1][0][wave - 1][lane] + sCD[1][1][wave - 1][lm];
    }
  }

  // sliding window over three planes of the row-folded values
  //   us = My . x (mass), t = My . m + da Ky . x (m = x, or T - Tp - dt f for RES)
  double us_m = 0.0, us_c = 0.0, t_m = 0.0, t_c = 0.0;
  double xc = 0.0;  // own-row value of the centre plane (p of the output node)
  double dot = 0.0, zz = 0.0, zr = 0.0;
  auto step = [&](int L, double c0, double c1, double h0, double h1, double pr, double pd) {
    const int buf = L & 1;
    double v, vm;
    combine(vo_own, L, c0, c1, v, vm);
    if (FUSEP) bstore(rsp, vo_wr + ((L >= q0 && L < q1) ? plane_off(L) : kBadOff), v);
    lds[0][buf][wave + 1][lane] = v;
    if (MODE == MODE_RES) lds[NA - 1][buf][wave + 1][lane] = vm;
    if (halo) {
      double hv, hvm;
      combine(vo_halo, L, h0, h1, hv, hvm);
      lds[0][buf][hslot][lane] = hv;
      if (MODE == MODE_RES) lds[NA - 1][buf][hslot][lane] = hvm;
    }
    __syncthreads();
    // the own row (x1) stays in registers; rows r - 1 and r + 1 from the slab
    const double x0 = lds[0][buf][wave][lane], x1 = v, x2 = lds[0][buf][wave + 2][lane];
    const double us_p = My0 * x0 + My1 * x1 + My2 * x2;
    const double vs_p = Ky0 * x0 + Ky1 * x1 + Ky2 * x2;
    double um_p = us_p;
    if (MODE == MODE_RES) um_p = My0 * lds[NA - 1][buf][wave][lane] + My1 * vm + My2 * lds[NA - 1][buf][wave + 2][lane];
    const double t_p = um_p + da * vs_p;
    if (L >= q0 + 1 && L <= q1) {
      const int q = L - 1;
      const double2* cq = cql[q - q0 + 1];
      const double2 c01 = cq[0], c23 = cq[1], c45 = cq[2], c67 = cq[3], c89 = cq[4];
      //   S1 = Mz . t + da Kz . us ,  S2 = da Mz . us          (march axis)
      const double S1 = c01.x * t_m + c01.y * t_c + c23.x * t_p + (c23.y * us_m + c45.x * us_c + c45.y * us_p);
      const double S2 = c67.x * us_m + c67.y * us_c + c89.x * us_p;
      // x axis by symmetry of the assembled 1D rows (Mlo_i = Mup_{i-1}, Klo_i = Kup_{i-1}):
      //   y_i = Mdi S1_i + Kdi S2_i + [Mup S1 + Kup S2]_{i-1} + [Mlo S1 + Klo S2]_{i+1}
      const double2 xlo = cxl[0][lane], xdi = cxl[1][lane], xup = cxl[2][lane];
      const double Lt = xup.x * S1 + xup.y * S2;
      const double Rt = xlo.x * S1 + xlo.y * S2;
      const double y = (xdi.x * S1 + xdi.y * S2) + (shr1(Lt) + shl1(Rt));
      const bool q_owned = (raxis == 2) ? true : (q >= kb && q < ke);
      const bool q_inwin = (raxis == 2) ? true : (q >= wb && q < we);
      const bool wr = writer && row_ok && row_owned && q_owned;  // records
      const bool inwin = row_inwin && q_inwin;                   // stores
      // Robin facet terms: in-tile face planes (above), face workgroups
      // (other faces, added by the consumer) / k_cg_boundary (residual)
      double yb = y;
      if (fq0 && q == 0) yb += yq0;
      if (fq1 && q == nQ - 1) yb += yq1;
      if (POST) {  // z = x + omega dinv (r - J x): the post-smoothing step (facet terms of the side faces later)
        // interior D^-1 from the staged coefficients (x pair, row SGPRs, plane slots 1 / 4 / 7 = Mz, da Kz, da Mz)
        const double xm = xdi.x, xk = xdi.y;
        const double dI = xm * My1 * c01.y + ((xk * My1 * c67.y + xm * Ky1 * c67.y) + xm * My1 * c45.x);
        const double dq = (bnd_lr || bnd_q(q)) ? pd : 1.0 / dI;
        const double zq = xc + pa.omega * dq * (pr - yb);
        bstore(rso, inwin ? vo_wr + plane_off(q) : kBadOff, zq);
        zz += wr ? zq * zq : 0.0;
        zr += wr ? zq * pr : 0.0;
      } else {
        bstore(rso, inwin ? vo_wr + plane_off(q) : kBadOff, yb);
      }
      if (MODE == MODE_JAC && !POST) dot += wr ? xc * yb : 0.0;
    }
    xc = x1;
    us_m = us_c; us_c = us_p;
    t_m = t_c; t_c = t_p;
  };
  // no early exits: steps past q1 only touch LDS (their stores are masked), so
  // the register sets keep fixed registers across the back edge
  for (int L = q0 - 1; L <= q1; L += PF + 1) {
#pragma unroll
    for (int s = 0; s <= PF; ++s) {
      const int sf = (s + PF) % (PF + 1);  // the set consumed one step ago
      fetch(vo_own, L + s + PF, ra0[sf], ra1[sf]);
      fetch(vo_halo, L + s + PF, rh0[sf], rh1[sf]);
      fetch_post(L + s + PF, rr[sf], rd[sf]);
      step(L + s, ra0[s], ra1[s], rh0[s], rh1[s], POST ? rr[s] : 0.0, POST ? rd[s] : 0.0);
    }
  }
  if (POST) {  // (z.z, z.r) records of the tile; k_mg_post_faces reduces them
    zz = wave_sum(zz);
    zr = wave_sum(zr);
    if (lane == 0) {
      red[wave] = zz;
      fsm[wave] = zr;  // the face LDS is free after the prologue
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      double a = 0.0, c = 0.0;
#pragma unroll
      for (int w = 0; w < R; ++w) {
        a += red[w];
        c += fsm[w];
      }
      store_partial(&partials[2 * (int64_t)bid], a);
      store_partial(&partials[2 * (int64_t)bid + 1], c);
    }
    return;
  }
  if (MODE == MODE_JAC && partials != nullptr) {
    dot = wave_sum(dot);
    if (lane == 0) red[wave] = dot;
    __syncthreads();
    if (threadIdx.x == 0) {
      double s = 0.0;
#pragma unroll
      for (int w = 0; w < R; ++w) s += red[w];
      store_partial(&partials[blockIdx.x], s);
    }
    fused_reduce_tail<1>(rt, nrec);  // p.w over all tiles (+ KSPCG logic, or the lagged state)
  }
}

// ---------------------------------------------------------------------------
// Single-reduction Jacobi-PCG iteration fused with the marching Jacobian: the
// Chronopoulos-Gear form of CG, ONE launch and ONE reduction per iteration
// (PETSc KSPCG, which the reference runs at ThermoViscoProblem.py:339-346,
// needs two: p.w for alpha, then z.r and z.z for beta and the norm test).
//
// Iteration i (i >= 1) with alpha = alpha_{i-1}, beta = beta_{i-1}, per node:
//     w_full = w_{i-1} + facet terms        (face workgroups' faces, f_{i-1})
//     s_{i-1} = w_full + beta s_{i-2}       (= A p_{i-1} by recurrence)
//     p_{i-1} = z_{i-1} + beta p_{i-2},  z_{i-1} = B r_{i-1}
//     x_i = x_{i-1} + alpha p_{i-1}
//     r_i = r_{i-1} - alpha s_{i-1},  z_i = B r_i      (B = diag(J)^-1)
//     w_i = J z_i                            (the march below)
//     partial sums (r_i, z_i), (z_i, w_i + facet terms), (z_i, z_i)
// and the tail turns the sums into gamma_i = (r, z), eta_i = delta_i -
// beta_i gamma_i / alpha_{i-1} (= (p_i, A p_i)), alpha_i, beta_i and PETSc's
// convergence test on ||z_i|| (KSPConvergedDefault, preconditioned norm): the
// same iterates as KSPCG in exact arithmetic.  i = 0 (INIT): z_0 = B r_0,
// w_0 = J z_0, x = 0.  At i = 1 p and s start as z_0 and w_0 (no beta term).
//
// z at the halo rows of a tile is recomputed from r, s, w (+ facet terms) and
// diag^-1 of the previous iteration, so r, s and w ping-pong between two
// buffers (neighbouring tiles read the old values while this launch writes
// the new ones); p and x are touched at owned nodes only, in place.  Loads,
// LDS exchange, sliding window, coefficient staging and the in-tile faces
// normal to the march axis follow k_cg_march.
// ---------------------------------------------------------------------------

// byte offset of the facet term of node (i, j, k) on the x faces / on the
// faces normal to storage axis ra (1 or 2) in the face buffer, or kBadOff
__device__ __forceinline__ uint32_t ff_off_x(const CgGrid& g, int i, int j, int k) {
  const int f = (i == 0) ? 0 : (i == g.n0 - 1 ? 1 : -1);
  if (f < 0 || g.ffoff[f] < 0) return kBadOff;
  return (uint32_t)(g.ffoff[f] + j + (int64_t)g.n1 * k) * 8u;
}
__device__ __forceinline__ uint32_t ff_off_r(const CgGrid& g, int ra, int i, int j, int k) {
  const int c = (ra == 1) ? j : k, n = (ra == 1) ? g.n1 : g.n2;
  const int side = (c == 0) ? 0 : (c == n - 1 ? 1 : -1);
  if (side < 0 || i < 0 || i >= g.n0) return kBadOff;
  const int f = 2 * ra + side;
  if (g.ffoff[f] < 0) return kBadOff;
  return (uint32_t)(g.ffoff[f] + i + (int64_t)g.n0 * ((ra == 1) ? k : j)) * 8u;
}

// the single-reduction scalars of iteration it (alpha_{i-1}, beta_{i-1})
struct CgsScal {
  double a, b;
  bool first;
};

// node update (see above); own = the node's p and x are updated too
template <bool INIT>
__device__ __forceinline__ void cgs_node(const CgsScal& k, double R, double S, double W, double D, double ff,
                                         double& s, double& r, double& u) {
  if (INIT) {
    s = 0.0;
    r = R;
  } else {
    const double wf = W + ff;
    s = k.first ? wf : wf + k.b * S;
    r = R - k.a * s;
  }
  u = D * r;
}

// Face workgroup of the single-reduction iteration: as face_block, with z_i
// recomputed at the staged face nodes from (r, s, w + f, diag^-1) of the
// previous iteration; writes f_i and the (0, z.f, 0) partial record.
template <bool INIT, int R>
__device__ void face_block_cgs(const CgGrid& g, const CgsBuffers& v, const CgsScal& ks, int raxis,
                               double* __restrict__ partials, int fb, const FaceOff& fo, double* sm,
                               double (*red)[R]) {
  double (*sT)[kWave] = reinterpret_cast<double (*)[kWave]>(sm);
  double (*sP)[kWave] = reinterpret_cast<double (*)[kWave]>(sm + (R + 1) * kWave);
  double (*sCD)[R][kWave] = reinterpret_cast<double (*)[R][kWave]>(sm + 2 * (R + 1) * kWave);
  int f = 0;
  while (f < 5 && fb >= fo.off[f + 1]) ++f;
  const int a = f >> 1, side = f & 1;
  const int t1 = (a == 0) ? 1 : 0, t2 = (a == 2) ? 1 : 2;
  const int n[3] = {g.n0, g.n1, g.n2};
  const int n1 = n[t1], n2 = n[t2];
  const int nseg1 = (n1 + kSeg - 1) / kSeg;
  const int tile = fb - fo.off[f];
  const int seg = tile % nseg1, tb = tile / nseg1;
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c1 = seg * kSeg - 1 + lane;
  const int r0 = tb * (R - 1);
  const bool ok1 = c1 >= 0 && c1 < n1;
  // T and z_i of one staged node; z_i from the previous iteration's r, s,
  // w + facet terms (x face, then row face: the order of the march's loads)
  // staging in two halves: the loads of every staged row first (wave R - 1
  // stages two; the facet terms by buffer loads with out-of-range offsets, not
  // loads under the face tests), then the arithmetic and the LDS stores
  const buf_t rsFin = mk_rsrc(v.fin, (uint32_t)(g.ffsize * 8));
  struct Stg {
    double tt, R_, D, S, W, fx, fr;
    bool ok;
  };
  auto stage_ld = [&](int cc2) -> Stg {
    Stg q{};
    q.ok = ok1 && cc2 >= 0 && cc2 < n2;
    int c[3];
    c[t1] = q.ok ? c1 : 0;
    c[t2] = q.ok ? cc2 : 0;
    c[a] = side ? n[a] - 1 : 0;
    const int64_t o = c[0] + (int64_t)g.n0 * c[1] + (int64_t)g.n0 * g.n1 * c[2];
    q.tt = v.T[o];
    q.R_ = v.rin[o];
    q.D = v.dinv[o];
    if (!INIT) {
      q.S = ks.first ? 0.0 : v.sin[o];
      q.W = v.win[o];
      q.fx = bload(rsFin, ff_off_x(g, c[0], c[1], c[2]));
      q.fr = bload(rsFin, ff_off_r(g, raxis, c[0], c[1], c[2]));
    }
    return q;
  };
  auto stage_st = [&](int row, const Stg& q) {
    double s, r, u;
    cgs_node<INIT>(ks, q.R_, q.S, q.W, q.D, INIT ? 0.0 : q.fx + q.fr, s, r, u);
    sT[row][lane] = q.ok ? q.tt : 0.0;
    sP[row][lane] = q.ok ? u : 0.0;
  };
  const int fr = r0 - 1 + wave;
  const bool facet_ok = c1 >= 0 && c1 < n1 - 1 && fr >= 0 && fr < n2 - 1;
  const double h1 = g.coef[t1][(int64_t)(facet_ok ? c1 : 0) * C_NCOEF + C_HHI];
  const double h2 = g.coef[t2][(int64_t)(facet_ok ? fr : 0) * C_NCOEF + C_HHI];
  const Stg sa = stage_ld(r0 - 1 + wave);
  Stg sb{};
  if (wave == R - 1) sb = stage_ld(r0 + R - 1);  // wave-uniform
  stage_st(wave, sa);
  if (wave == R - 1) stage_st(R, sb);
  __syncthreads();
  const double Pa = sP[wave][lane];
  double ya, yb, yc, yd;
  facet_corners(g, facet_ok, h1, h2, sT[wave][lane], sT[wave + 1][lane], Pa, sP[wave + 1][lane], ya, yb, yc, yd);
  sCD[0][wave][lane] = yc;
  sCD[1][wave][lane] = yd;
  const double ybl = shr1(yb);
  __syncthreads();
  double dot = 0.0;
  const int c2 = r0 - 1 + wave;
  const bool wr = wave >= 1 && ok1 && lane >= 1 && lane <= kSeg && c2 < n2;
  if (wr) {
    const double acc = (ya + ybl) + (sCD[0][wave - 1][lane] + sCD[1][wave - 1][lane - 1]);
    int c[3];
    c[t1] = c1;
    c[t2] = c2;
    c[a] = side ? n[a] - 1 : 0;
    const bool owned = c[2] >= g.k_begin && c[2] < g.k_end;
    v.fout[g.ffoff[f] + c1 + (int64_t)n1 * c2] = owned ? acc : 0.0;
    dot = owned ? Pa * acc : 0.0;
  }
  dot = wave_sum(dot);
  if (lane == 0) red[1][wave] = dot;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s2 = 0.0;
#pragma unroll
    for (int w = 0; w < R; ++w) s2 += red[1][w];
    store_partial(&partials[(int64_t)blockIdx.x * 3 + 0], 0.0);
    store_partial(&partials[(int64_t)blockIdx.x * 3 + 1], s2);
    store_partial(&partials[(int64_t)blockIdx.x * 3 + 2], 0.0);
  }
}

template <bool INIT, int R, int PF>
__global__ __launch_bounds__(R * kWave) void k_cgs_march(CgGrid g, CgsBuffers v, PcgState* __restrict__ st,
                                                         double* __restrict__ partials, int nseg, int raxis,
                                                         int qchunk, RedTail rt, int nrec, int nmarch, FaceOff fo,
                                                         int it_host, const double* __restrict__ lag_sums) {
  stamp_start(rt);
  __shared__ double lds[2][R + 2][kWave];  // double-buffered plane slab of z
  __shared__ double red[3][R];
  constexpr int kFaceLds = (8 * R + 8) * kWave;
  __shared__ double fsm[kFaceLds];
  __shared__ PcgState sst;  // lagged mode: this launch's view of the state
  // ---- scalars: alpha_{i-1}, beta_{i-1} ----------------------------------------
  CgsScal ks{0.0, 0.0, it_host == 1};
  int st_done = 0;
  if (lag_sums != nullptr) {
    // multi-rank: the state after the previous iteration is formed here from
    // the all-reduced sums (identically in every workgroup); committed by WG 0
    // when it ends the solve, else by this launch's tail
    if (threadIdx.x == 0) {
      sst = *st;
      apply_logic(&sst, lag_sums, it_host == 1 ? 4 : 5);
    }
    __syncthreads();
    if (sst.done) {
      if (blockIdx.x == 0 && threadIdx.x == 0 && !st->done) *st = sst;
      return;
    }
    ks.a = sst.a;
    ks.b = sst.beta;
  } else if (!INIT) {
    // converged: every launch queued behind exits -- tested once the block's
    // first loads are in flight (scalar loads, issued here)
    st_done = st->done;
    ks.a = st->a;
    ks.b = st->beta;
  }
  const int nface = (int)gridDim.x - nmarch;
  if ((int)blockIdx.x >= nmarch && nface > 0) {
    if (st_done) return;
    face_block_cgs<INIT, R>(g, v, ks, raxis, partials, (int)blockIdx.x - nmarch, fo, fsm, red);
    cgs_tail(rt, nrec, st, lag_sums != nullptr ? &sst : nullptr);
    return;
  }
  const int lane = threadIdx.x & (kWave - 1);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int n0 = g.n0;
  const int nR = (raxis == 1) ? g.n1 : g.n2;
  const int nQ = (raxis == 1) ? g.n2 : g.n1;
  const int64_t sR = (raxis == 1) ? (int64_t)n0 : (int64_t)n0 * g.n1;
  const int64_t sQ = (raxis == 1) ? (int64_t)n0 * g.n1 : (int64_t)n0;
  // tile order as k_cg_march: x segment fastest, then row block, then chunk
  const int nrbk = (nR + R - 1) / R;
  int seg, rb, chunk;  // face-chunk tiles spread over the XCDs, first (march_tile)
  march_tile((int)blockIdx.x, nmarch, nseg, nrbk, (nQ + qchunk - 1) / qchunk, seg, rb, chunk);
  const int r0 = rb * R;
  const int r = r0 + wave;
  const bool row_ok = r < nR;
  const int q0 = chunk * qchunk;
  const int q1 = min(q0 + qchunk, nQ);
  const int i = seg * kSeg - 1 + lane;
  const bool col_ok = (i >= 0) && (i < n0);
  const bool writer = col_ok && lane >= 1 && lane <= kSeg;
  const int kb = g.k_begin, ke = g.k_end;
  const bool row_owned = (raxis == 2) ? (r >= kb && r < ke) : true;

  // per-axis data by selects (as k_cg_march)
  const double* coefR = (raxis == 1) ? g.coef[1] : g.coef[2];
  const double* coefQ = (raxis == 1) ? g.coef[2] : g.coef[1];
  const int bq_lo = (raxis == 1) ? g.bnd[2][0] : g.bnd[1][0];
  const int bq_hi = (raxis == 1) ? g.bnd[2][1] : g.bnd[1][1];
  const bool fq0 = q0 == 0 && bq_lo;
  const bool fq1 = q1 == nQ && bq_hi;
  double (*sFq)[2][R + 2][kWave] = reinterpret_cast<double (*)[2][R + 2][kWave]>(fsm);
  double (*sCD)[2][R][kWave] = reinterpret_cast<double (*)[2][R][kWave]>(fsm + 4 * (R + 2) * kWave);
  double yq0 = 0.0, yq1 = 0.0;
  const double da = g.dt_alpha;

  // ---- buffer descriptors (out-of-range offsets read 0 / drop the store) -----
  const uint32_t nbytes = (uint32_t)g.n0 * (uint32_t)g.n1 * (uint32_t)g.n2 * 8u;
  const buf_t rsR = mk_rsrc(v.rin, nbytes);
  const buf_t rsD = mk_rsrc(v.dinv, nbytes);
  const buf_t rsS = mk_rsrc(v.sin, (INIT || ks.first) ? 0u : nbytes);
  const buf_t rsW = mk_rsrc(v.win, INIT ? 0u : nbytes);
  const buf_t rsF = mk_rsrc(v.fin, INIT ? 0u : (uint32_t)g.ffsize * 8u);
  const buf_t rsP = mk_rsrc(v.p, (INIT || ks.first) ? 0u : nbytes);
  const buf_t rsX = mk_rsrc(v.x, (INIT || ks.first) ? 0u : nbytes);
  const buf_t wsR = mk_rsrc(v.rout, INIT ? 0u : nbytes);
  const buf_t wsS = mk_rsrc(v.sout, INIT ? 0u : nbytes);
  const buf_t wsP = mk_rsrc(v.p, INIT ? 0u : nbytes);
  const buf_t wsX = mk_rsrc(v.x, nbytes);  // INIT: x = 0
  const buf_t wsW = mk_rsrc(v.wout, nbytes);
  const buf_t rsT = mk_rsrc(v.T, (fq0 || fq1) ? nbytes : 0u);
  const bool halo = (wave == 0) || (wave == R - 1);
  const int hrow = (wave == 0) ? r0 - 1 : (wave == R - 1 ? r0 + R : r);
  const int hslot = (wave == 0) ? 0 : R + 1;
  auto lane_off = [&](int rr) -> uint32_t {
    return (col_ok && rr >= 0 && rr < nR) ? (uint32_t)(i + sR * rr) * 8u : kBadOff;
  };
  const uint32_t vo_own = lane_off(r), vo_halo = halo ? lane_off(hrow) : kBadOff;
  const uint32_t vo_wr = writer ? vo_own : kBadOff;
  auto plane_off = [&](int L) -> uint32_t { return (L >= 0 && L < nQ) ? (uint32_t)(sQ * L) * 8u : kBadOff; };
  // facet terms of the face-workgroup faces at (i, row rr, plane L): x face,
  // then the face normal to the row axis (base offsets per row, per lane)
  auto xf_base = [&](int rr) -> int64_t {
    if (!col_ok || rr < 0 || rr >= nR) return -1;
    const int f = (i == 0) ? 0 : (i == n0 - 1 ? 1 : -1);
    return (f < 0) ? -1 : g.ffoff[f];
  };
  auto rf_base = [&](int rr) -> int64_t {
    if (!col_ok) return -1;
    const int f = (rr == 0) ? 2 * raxis : (rr == nR - 1 ? 2 * raxis + 1 : -1);
    return (f < 0) ? -1 : g.ffoff[f];
  };
  const int64_t xb_own = xf_base(r), rb_own = rf_base(r);
  const int64_t xb_hal = halo ? xf_base(hrow) : -1, rb_hal = halo ? rf_base(hrow) : -1;
  auto ff_offs = [&](int64_t xb, int64_t rbse, int rr, int L, uint32_t& ox, uint32_t& orr) {
    const bool okL = L >= 0 && L < nQ;
    const int64_t ix = (raxis == 2) ? ((int64_t)L + (int64_t)g.n1 * rr) : ((int64_t)rr + (int64_t)g.n1 * L);
    ox = (xb >= 0 && okL) ? (uint32_t)(xb + ix) * 8u : kBadOff;
    orr = (rbse >= 0 && okL) ? (uint32_t)(rbse + i + (int64_t)n0 * L) * 8u : kBadOff;
  };

  // raw loads of one (row, plane): r, s, w, diag^-1, facet terms (x, row)
  struct Raw { double Rv, Sv, Wv, Dv, FX, FR, Pv, Xv; };
  auto fetch = [&](uint32_t vo, int64_t xb, int64_t rbse, int rr, int L, Raw& a, bool own) {
    const uint32_t o = vo + plane_off(L);
    a.Rv = bload(rsR, o);
    a.Dv = bload(rsD, o);
    a.Pv = a.Xv = 0.0;
    if (!INIT && own) {
      a.Pv = bload(rsP, o);
      a.Xv = bload(rsX, o);
    }
    if (!INIT) {
      a.Sv = bload(rsS, o);
      a.Wv = bload(rsW, o);
      uint32_t ox, orr;
      ff_offs(xb, rbse, rr, L, ox, orr);
      a.FX = bload(rsF, ox);
      a.FR = bload(rsF, orr);
    } else {
      a.Sv = a.Wv = a.FX = a.FR = 0.0;
    }
  };
  Raw ra[PF + 1], rh[PF + 1] = {};
#pragma unroll
  for (int sI = 0; sI < PF; ++sI) {
    fetch(vo_own, xb_own, rb_own, r, q0 - 1 + sI, ra[sI], true);
    if (halo) fetch(vo_halo, xb_hal, rb_hal, hrow, q0 - 1 + sI, rh[sI], false);
  }
  // coefficient stages (march axis, x axis, the tile's rows; as k_cg_march),
  // issued with the prefetch
  __shared__ double2 cql[kFaceChunk + 2][5];
  __shared__ double2 cxl[4][kWave];
  __shared__ double crl[R + 1][C_NCOEF];
  const int nqs = q1 - q0 + 2;
  const bool st_q = (int)threadIdx.x < nqs * 6;
  const bool st_x = (int)threadIdx.x < 8 * kWave;
  const bool st_r = (int)threadIdx.x < (R + 1) * C_NCOEF;
  double cqv, cxv, crv;
  {
    const int e = threadIdx.x;
    const int qq = q0 - 1 + e / 6;
    const bool okq = st_q && qq >= 0 && qq < nQ;
    cqv = coefQ[okq ? (int64_t)qq * C_NCOEF + e % 6 : 0];
    const int ii = seg * kSeg - 1 + (e & (kWave - 1));
    const bool okx = st_x && ii >= 0 && ii < n0;
    const int k = e >> 6;
    const int cc = k == 0 ? C_MLO : k == 1 ? C_KLO : k == 2 ? C_MDI : k == 3 ? C_KDI : k == 4 ? C_MUP : k == 5 ? C_KUP : C_HHI;
    cxv = g.coef[0][okx ? (int64_t)ii * C_NCOEF + cc : 0];
    const int rrow = r0 - 1 + e / C_NCOEF;
    const bool okr = st_r && rrow >= 0 && rrow < nR;
    crv = coefR[okr ? (int64_t)rrow * C_NCOEF + e % C_NCOEF : 0];
    cqv = okq ? cqv : 0.0;
    cxv = (okx && k < 7) ? cxv : 0.0;
    crv = okr ? crv : 0.0;
  }
  if (st_done) return;
  // face planes normal to the march axis: T and z of the own and halo rows
  double fT[2][2], fU[2][2];
  if (fq0 || fq1) {
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      const int Lf = f == 0 ? (fq0 ? 0 : -1) : (fq1 ? nQ - 1 : -1);
      const uint32_t po = plane_off(Lf);
      fT[f][0] = bload(rsT, vo_own + po);
      fT[f][1] = bload(rsT, vo_halo + po);
      Raw a0, a1;
      fetch(vo_own, xb_own, rb_own, r, Lf, a0, false);
      fetch(vo_halo, xb_hal, rb_hal, hrow, Lf, a1, false);
      double s_, r_;
      cgs_node<INIT>(ks, a0.Rv, a0.Sv, a0.Wv, a0.Dv, a0.FX + a0.FR, s_, r_, fU[f][0]);
      cgs_node<INIT>(ks, a1.Rv, a1.Sv, a1.Wv, a1.Dv, a1.FX + a1.FR, s_, r_, fU[f][1]);
    }
  }
  if (st_q) {
    const int qs = threadIdx.x / 6, c = threadIdx.x % 6;
    double* row = reinterpret_cast<double*>(cql[qs]);
    if (c < 3) {
      row[c] = cqv;
      row[6 + c] = da * cqv;
    } else {
      row[c] = da * cqv;
    }
    if (c == 0) row[9] = 0.0;
  }
  if (st_x) reinterpret_cast<double*>(cxl[(threadIdx.x >> 6) >> 1])[2 * (threadIdx.x & (kWave - 1)) + ((threadIdx.x >> 6) & 1)] = cxv;
  if (st_r) crl[threadIdx.x / C_NCOEF][threadIdx.x % C_NCOEF] = crv;
  if (fq0 || fq1) {
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      sFq[f][0][wave + 1][lane] = fT[f][0];
      sFq[f][1][wave + 1][lane] = fU[f][0];
      if (halo) {
        sFq[f][0][hslot][lane] = fT[f][1];
        sFq[f][1][hslot][lane] = fU[f][1];
      }
    }
  }
  __syncthreads();
  // row coefficients, wave-uniform in SGPRs (row slot wave + 1)
  const double* crw = crl[wave + 1];
  const double My0 = uniform(crw[C_MLO]), My1 = uniform(crw[C_MDI]), My2 = uniform(crw[C_MUP]);
  const double Ky0 = uniform(crw[C_KLO]), Ky1 = uniform(crw[C_KDI]), Ky2 = uniform(crw[C_KUP]);
  const double hq_own = uniform(crw[C_HHI]);
  const double hq_low = uniform(crl[0][C_HHI]);
  if (fq0 || fq1) {
    const bool cok = i >= 0 && i < n0 - 1;
    const double h1 = cxl[3][lane].x;
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      if (!(f == 0 ? fq0 : fq1)) continue;
      double ya, yb, yc, yd;
      facet_corners(g, cok && r < nR - 1, h1, hq_own, sFq[f][0][wave + 1][lane], sFq[f][0][wave + 2][lane],
                    sFq[f][1][wave + 1][lane], sFq[f][1][wave + 2][lane], ya, yb, yc, yd);
      double yq = ya + shr1(yb);
      sCD[f][0][wave][lane] = yc;
      sCD[f][1][wave][lane] = yd;
      if (wave == 0) {
        facet_corners(g, cok && r0 >= 1 && r0 - 1 < nR - 1, h1, hq_low, sFq[f][0][0][lane], sFq[f][0][1][lane],
                      sFq[f][1][0][lane], sFq[f][1][1][lane], ya, yb, yc, yd);
        yq += yc + shr1(yd);
      }
      if (f == 0) yq0 = yq; else yq1 = yq;
    }
    __syncthreads();
    if (wave >= 1) {
      const int lm = lane >= 1 ? lane - 1 : 0;
      yq0 += sCD[0][0][wave - 1][lane] + sCD[0][1][wave - 1][lm];
      yq1 += sCD[1][0][wave - 1][lane] + sCD[1][1][wave - 1][lm];
    }
  }

  // ---- the march ----------------------------------------------------------------
  double us_m = 0.0, us_c = 0.0, t_m = 0.0, t_c = 0.0;
  double uc = 0.0, rc = 0.0;  // z_i and r_i of the centre plane (output node)
  double dg = 0.0, dd = 0.0, dn = 0.0;  // partial (r, z), (z, w), (z, z)
  auto step = [&](int L, const Raw& a, const Raw& h) {
    const int buf = L & 1;
    const bool qin = (L >= q0 && L < q1);
    const uint32_t po = qin ? plane_off(L) : kBadOff;
    double s, rr, u;
    cgs_node<INIT>(ks, a.Rv, a.Sv, a.Wv, a.Dv, a.FX + a.FR, s, rr, u);
    // own row: r, s (every local node incl. ghost planes), p, x (owned nodes)
    const bool own_n = row_owned && ((raxis == 2) ? true : (L >= kb && L < ke));
    if (!INIT) {
      bstore(wsR, vo_wr + po, rr);
      bstore(wsS, vo_wr + po, s);
    }
    {
      const uint32_t o = vo_wr + (own_n ? po : kBadOff);
      if (INIT) {
        bstore(wsX, o, 0.0);
      } else {
        const double uo = a.Dv * a.Rv;  // z_{i-1}
        const double Pv = ks.first ? uo : uo + ks.b * a.Pv;
        const double Xv = ks.first ? ks.a * Pv : a.Xv + ks.a * Pv;
        bstore(wsP, o, Pv);
        bstore(wsX, o, Xv);
      }
    }
    lds[buf][wave + 1][lane] = u;
    if (halo) {
      double hs, hr, hu;
      cgs_node<INIT>(ks, h.Rv, h.Sv, h.Wv, h.Dv, h.FX + h.FR, hs, hr, hu);
      lds[buf][hslot][lane] = hu;
    }
    __syncthreads();
    const double x0 = lds[buf][wave][lane], x1 = u, x2 = lds[buf][wave + 2][lane];
    const double us_p = My0 * x0 + My1 * x1 + My2 * x2;
    const double vs_p = Ky0 * x0 + Ky1 * x1 + Ky2 * x2;
    const double t_p = us_p + da * vs_p;
    if (L >= q0 + 1 && L <= q1) {
      const int q = L - 1;
      const double2* cq = cql[q - q0 + 1];
      const double2 c01 = cq[0], c23 = cq[1], c45 = cq[2], c67 = cq[3], c89 = cq[4];
      const double S1 = c01.x * t_m + c01.y * t_c + c23.x * t_p + (c23.y * us_m + c45.x * us_c + c45.y * us_p);
      const double S2 = c67.x * us_m + c67.y * us_c + c89.x * us_p;
      const double2 xlo = cxl[0][lane], xdi = cxl[1][lane], xup = cxl[2][lane];
      const double Lt = xup.x * S1 + xup.y * S2;
      const double Rt = xlo.x * S1 + xlo.y * S2;
      const double y = (xdi.x * S1 + xdi.y * S2) + (shr1(Lt) + shl1(Rt));
      const bool q_owned = (raxis == 2) ? true : (q >= kb && q < ke);
      const bool wr = writer && row_ok && row_owned && q_owned;
      double yb = y;
      if (fq0 && q == 0) yb += yq0;
      if (fq1 && q == nQ - 1) yb += yq1;
      bstore(wsW, (row_owned && q_owned) ? vo_wr + plane_off(q) : kBadOff, yb);
      if (wr) {
        dg += rc * uc;
        dd += uc * yb;
        dn += uc * uc;
      }
    }
    uc = u;
    rc = rr;
    us_m = us_c; us_c = us_p;
    t_m = t_c; t_c = t_p;
  };
  for (int L = q0 - 1; L <= q1; L += PF + 1) {
#pragma unroll
    for (int sI = 0; sI <= PF; ++sI) {
      const int sf = (sI + PF) % (PF + 1);
      fetch(vo_own, xb_own, rb_own, r, L + sI + PF, ra[sf], true);
      if (halo) fetch(vo_halo, xb_hal, rb_hal, hrow, L + sI + PF, rh[sf], false);  // waves 0 and R-1 only
      step(L + sI, ra[sI], rh[sI]);
    }
  }
  // ---- partial record (r.z, z.w, z.z) + tail ------------------------------------
  dg = wave_sum(dg);
  dd = wave_sum(dd);
  dn = wave_sum(dn);
  if (lane == 0) {
    red[0][wave] = dg;
    red[1][wave] = dd;
    red[2][wave] = dn;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int w3 = 0; w3 < 3; ++w3) {
      double s3 = 0.0;
#pragma unroll
      for (int w = 0; w < R; ++w) s3 += red[w3][w];
      store_partial(&partials[(int64_t)blockIdx.x * 3 + w3], s3);
    }
  }
  cgs_tail(rt, nrec, st, lag_sums != nullptr ? &sst : nullptr);
}

// Robin facet terms of the owned boundary nodes (list built at context
// creation), added after the marching kernel: out[n] += dt * sum_f int_f ...,
// and the matching p.w correction for the PCG dot product.  For the fused PCG
// matvec the input is the freshly written p (buffer selected from st->it).
template <int MODE, bool FUSEP>
// dinv != nullptr (residual of the Newton loop): also the inverse Jacobian
// diagonal at the boundary nodes for the same T (k_cg_diag_bnd's work, one
// launch fewer per Newton iteration)
__global__ __launch_bounds__(kBlock) void k_cg_boundary(CgGrid g, const int64_t* __restrict__ bnodes, int64_t nb,
                                                        const double* __restrict__ T, const double* in0,
                                                        const double* pB, double* __restrict__ out,
                                                        const PcgState* __restrict__ st,
                                                        double* __restrict__ partials, double* __restrict__ dinv) {
  __shared__ double red[kBlock / kWave];
  if (FUSEP && st->done) return;
  const double* x = in0;
  if (FUSEP) x = (st->it & 1) ? pB : in0;
  double dot = 0.0;
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < nb; t += (int64_t)gridDim.x * kBlock) {
    const int64_t n = bnodes[t];
    int i, j, k;
    decode_node(n, g, i, j, k);
    const int c[3] = {i, j, k};
    const int nn[3] = {g.n0, g.n1, g.n2};
    double acc = 0.0;
#pragma unroll 1
    for (int a = 0; a < 3; ++a) {
      if ((c[a] == 0 && g.bnd[a][0]) || (c[a] == nn[a] - 1 && g.bnd[a][1]))
        acc += facet_direct<MODE, false>(g, i, j, k, a, T, x, nullptr, 0.0, true);
    }
    out[n] += acc;
    if (MODE == MODE_JAC) dot += x[n] * acc;
    if (MODE == MODE_RES && dinv != nullptr) dinv[n] = 1.0 / diag_value<3, true>(g, T, n);
  }
  if (MODE == MODE_JAC && partials != nullptr) {
    dot = wave_sum(dot);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) red[wave] = dot;
    __syncthreads();
    if (threadIdx.x == 0) store_partial(&partials[blockIdx.x], (red[0] + red[1]) + (red[2] + red[3]));
  }
}


int dim_of(const CgGrid& g) { return g.deg2 ? 1 : (g.deg1 ? 2 : 3); }

// march chunking: split the march axis until the grid has kMarchMinBlocks
// tiles (256 CUs x 4), down to kMarchMinQ planes per chunk; tiny grids further
constexpr int kMarchMinBlocks = 1024;  // 512: the same at C4, 2048: 7 % slower (measured)
constexpr int kMarchMinQ = 6;  // 3 / 4: the same at C4, 1-3 % slower at C3 (measured)
constexpr int kMarchSmallTiles = 256;  // one marching tile per CU

struct Launch {
  int blocks, nseg, kfirst, nplanes, wmode, rows;
  int nparts;  // partial records written (JAC)
  bool march;
  int raxis, qchunk;
};

bool use_march(const CgGrid& g) {
  // the marching kernel addresses the fields with 32-bit buffer offsets
  const int64_t bytes = (int64_t)g.n0 * g.n1 * g.n2 * 8;
  return dim_of(g) == 3 && bytes < (int64_t)kBadOff;
}

int bnd_blocks(const CgGrid& g) {
  int64_t b = (g.n_bnodes + kBlock - 1) / kBlock;
  return (int)std::max<int64_t>(1, std::min<int64_t>(b, 1024));
}

Launch plan(const CgGrid& g, bool ghosts) {
  Launch L{};
  L.nseg = (g.n0 + kSeg - 1) / kSeg;
  L.march = use_march(g);
  if (L.march) {
    // rows along the longer of storage axes 1/2, march along the shorter one;
    // the kernel covers every local node (ghost planes included) so the fused
    // PCG matvec refreshes p everywhere; outputs go to owned nodes only.
    L.raxis = (g.n2 >= g.n1) ? 2 : 1;
    L.rows = kRows;
    const int nR = (L.raxis == 1) ? g.n1 : g.n2;
    const int nQ = (L.raxis == 1) ? g.n2 : g.n1;
    const int nrb = (nR + L.rows - 1) / L.rows;
    // enough workgroups to fill 256 CUs x ~4: split the march into chunks
    int nchunks = 1;
    while ((int64_t)L.nseg * nrb * nchunks < kMarchMinBlocks && nQ / (nchunks * 2) >= kMarchMinQ) nchunks *= 2;
    // tiny grids (fewer tiles than CUs): the march is a chain of plane steps, so
    // shorter chunks down to 2 planes (C2 100x100x10: 26 -> 104 tiles, fused
    // matvec 15.7 -> 10.1 us, step 1.29 -> 1.08 ms; measured)
    while ((int64_t)L.nseg * nrb * nchunks < kMarchSmallTiles && nQ / (nchunks * 2) >= 2) nchunks *= 2;
    while ((nQ + nchunks - 1) / nchunks > kFaceChunk) ++nchunks;  // LDS coefficient stage bound
    L.qchunk = (nQ + nchunks - 1) / nchunks;
    nchunks = (nQ + L.qchunk - 1) / L.qchunk;
    L.blocks = L.nseg * nrb * nchunks;
    // Jacobian partial records: one per marching tile and face workgroup
    L.nparts = L.blocks + face_offsets(g, L.rows, 3 - L.raxis).off[6];
    return L;
  }
  L.kfirst = ghosts ? g.k_begin - g.g_lo : g.k_begin;
  L.nplanes = (g.k_end - g.k_begin) + (ghosts ? g.g_lo + g.g_hi : 0);
  L.wmode = (g.n1 >= 4) ? 0 : 1;
  if (L.wmode == 0) {
    L.blocks = L.nseg * ((g.n1 + 3) / 4) * L.nplanes;
  } else {
    const int64_t waves = (int64_t)L.nseg * g.n1 * L.nplanes;
    L.blocks = (int)((waves + 3) / 4);
  }
  L.nparts = L.blocks;
  return L;
}

template <int MODE, bool FUSEP>
bool launch_rows(const CgGrid& g, const double* T, const double* in0, const double* in1, double* out,
                 double* pout, const PcgState* st, double* partials, bool ghosts, hipStream_t s,
                 const RedTail* tail = nullptr, int it_host = 0, bool addfaces = true, double* dinv_bnd = nullptr) {
  const Launch L = plan(g, ghosts);
  if (L.blocks <= 0) return false;
  if (L.march) {
    // Jacobian: the Robin facet terms come from k_cg_faces (launched first)
    // and are added inside the marching launch, which also runs the p.w
    // reduction tail
    const bool folded = MODE == MODE_JAC;
    RedTail rt{};
    if (folded && tail && partials) rt = *tail;
    const FaceOff fo = folded ? face_offsets(g, L.rows, 3 - L.raxis) : FaceOff{};
    const int grid = L.blocks + fo.off[6];
    // R = 8 rows, prefetch depth 2 (measured best, round 1-2: R = 16, PF 3 / 4,
    // 8 waves per SIMD and an LDS-DMA plane ring were all slower)
    hipLaunchKernelGGL((k_cg_march<MODE, FUSEP, kRows, 1, 2>), dim3(grid), dim3(kRows * kWave), 0, s, g, T, in0, in1,
                       out, pout, st, partials, L.nseg, L.raxis, L.qchunk, rt, L.nparts, L.blocks, fo, it_host,
                       PostArgs{});
    if (folded && !FUSEP && addfaces && fo.off[6] > 0) {  // complete J x (else the consumer adds them)
      const int64_t nodes = 2 * ((int64_t)g.n1 * (g.w_end - g.w_begin) + (int64_t)g.n0 * std::max(g.n1, g.n2));
      const int nb = (int)std::max<int64_t>(1, std::min<int64_t>((nodes + kBlock - 1) / kBlock, 1024));
      hipLaunchKernelGGL(k_cg_addfaces, dim3(nb), dim3(kBlock), 0, s, g, out, L.raxis, st);
    }
    if (folded) return rt.counter != nullptr;
    if (g.n_bnodes > 0) {
      hipLaunchKernelGGL((k_cg_boundary<MODE, FUSEP>), dim3(bnd_blocks(g)), dim3(kBlock), 0, s, g, g.bnodes,
                         g.n_bnodes, T, FUSEP ? in1 : in0, pout, out, st,
                         partials ? partials + L.blocks : nullptr, dinv_bnd);
    }
    return false;
  }
  switch (dim_of(g)) {
    case 1:
      hipLaunchKernelGGL((k_cg_rows<1, MODE, FUSEP>), dim3(L.blocks), dim3(kBlock), 0, s, g, T, in0, in1, out,
                         pout, st, partials, L.nseg, L.kfirst, L.nplanes, L.wmode);
      break;
    case 2:
      hipLaunchKernelGGL((k_cg_rows<2, MODE, FUSEP>), dim3(L.blocks), dim3(kBlock), 0, s, g, T, in0, in1, out,
                         pout, st, partials, L.nseg, L.kfirst, L.nplanes, L.wmode);
      break;
    default:
      hipLaunchKernelGGL((k_cg_rows<3, MODE, FUSEP>), dim3(L.blocks), dim3(kBlock), 0, s, g, T, in0, in1, out,
                         pout, st, partials, L.nseg, L.kfirst, L.nplanes, L.wmode);
  }
  return false;
}

// Facet terms of the face-workgroup faces (normal to storage axis 0 and to the
// row axis) for the POST march: z <- z - omega dinv (facet terms) at those
// nodes, and the changes of z.z and z.r as records rec0 + block (the march
// tiles wrote records 0 .. rec0 - 1); the last block reduces all of them and
// runs the KSPCG logic.  Nodes on both face families are visited once (the
// row-axis faces skip i = 0 and i = n0 - 1; face_at sums every face of a node).
// [kb, ke): the owned planes of storage axis 2, the only ones counted; z is
// rewritten on the write window [wb, we) (the owned planes, or on a deep-ghost
// slab every ghost plane but the outermost, where the single-reduction form
// needs z one plane out)
__global__ __launch_bounds__(kBlock) void k_mg_post_faces(FaceAdd fa, int raxis, const double* __restrict__ r,
                                                         const double* __restrict__ dinv, double omega,
                                                         double* __restrict__ z, double* __restrict__ partials,
                                                         int rec0, RedTail rt, const PcgState* __restrict__ st, int kb,
                                                         int ke, int wb, int we) {
  if (st->done) return;  // uniform: a converged solve's queued launch
  const int n0 = fa.n0, n1 = fa.n1, n2 = fa.n2;
  const int64_t nA = 2 * (int64_t)n1 * n2;
  const int nO = (raxis == 2) ? n1 : n2;  // the free axis of the row-axis faces besides x
  const int64_t nB = 2 * (int64_t)(n0 - 2) * nO;
  double a0 = 0.0, a1 = 0.0;
  const FaceRsrc fr = face_rsrc(fa);  // the face terms with the node's loads (a load under each face test waited at once)
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < nA + nB; t += (int64_t)gridDim.x * kBlock) {
    int i, j, k;
    if (t < nA) {
      const int64_t pl = (int64_t)n1 * n2;
      const int side = (int)(t / pl);
      const int64_t e = t - side * pl;
      i = side ? n0 - 1 : 0;
      j = (int)(e % n1);
      k = (int)(e / n1);
    } else {
      const int64_t u = t - nA, pl = (int64_t)(n0 - 2) * nO;
      const int side = (int)(u / pl);
      const int64_t e = u - side * pl;
      i = 1 + (int)(e % (n0 - 2));
      const int o = (int)(e / (n0 - 2));
      if (raxis == 2) {
        j = o;
        k = side ? n2 - 1 : 0;
      } else {
        k = o;
        j = side ? n1 - 1 : 0;
      }
    }
    if (k < wb || k >= we) continue;  // outside the write window
    const int64_t q = i + (int64_t)n0 * (j + (int64_t)n1 * k);
    // the node's three loads first, independent of the face lookups (one round trip)
    const double zo = z[q], dq = dinv[q], rq = r[q];
    const double add = face_at_nb(fa, fr, i, j, k);
    const double zn = zo - omega * dq * add;
    z[q] = zn;
    if (k < kb || k >= ke) continue;  // a ghost plane: rewritten, not counted
    a0 += zn * zn - zo * zo;
    a1 += (zn - zo) * rq;
  }
  __shared__ double red[2][kBlock / kWave];
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x >> 6;
  a0 = wave_sum(a0);
  a1 = wave_sum(a1);
  if (lane == 0) {
    red[0][wave] = a0;
    red[1][wave] = a1;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    const int w = threadIdx.x;
    store_partial(&partials[2 * ((int64_t)rec0 + blockIdx.x) + w], (red[w][0] + red[w][1]) + (red[w][2] + red[w][3]));
  }
  fused_reduce_tail<2>(rt, rec0 + (int)gridDim.x);
}

// Injection of every coarse level straight from the base level (nested grids:
// coarse node I of a level is fine node ri[3 I + 1] of the level above).  The
// level of a thread is wave-uniform (64-padded ranges).
__global__ __launch_bounds__(kBlock) void k_mg_prep_inject(MgPrep p) {
  const int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x;
  int l = 0;
  while (l + 1 < p.nlev && t >= p.off_n[l + 1]) ++l;
  l = __builtin_amdgcn_readfirstlane(l);
  const MgXfer& x = p.xf[l];
  const int64_t e = t - p.off_n[l];
  const int64_t nc = (int64_t)x.cn[0] * x.cn[1] * x.cn[2];
  if (e >= nc) return;
  int c0 = (int)(e % x.cn[0]);
  int c1 = (int)((e / x.cn[0]) % x.cn[1]);
  int c2 = (int)(e / ((int64_t)x.cn[0] * x.cn[1]));
  for (int m = l; m >= 0; --m) {  // down to the base level
    const MgXfer& y = p.xf[m];
    c0 = y.ri[0][3 * c0 + 1];
    c1 = y.ri[1][3 * c1 + 1];
    c2 = y.ri[2][3 * c2 + 1];
  }
  const MgXfer& b = p.xf[0];
  p.T[l][e] = p.Tbase[c0 + (int64_t)b.fn[0] * (c1 + (int64_t)b.fn[1] * c2)];
}

__global__ __launch_bounds__(kBlock) void k_mg_prep_diag(MgPrep p) {
  const int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x;
  int l = 0;
  while (l + 1 < p.nlev && t >= p.off_b[l + 1]) ++l;
  l = __builtin_amdgcn_readfirstlane(l);
  const CgGrid& g = p.g[l];
  const int64_t e = t - p.off_b[l];
  if (e >= g.n_bnodes) return;
  const int64_t n = g.bnodes[e];
  p.dinv[l][n] = 1.0 / diag_value<3, true>(g, p.T[l], n);
}


// Robin facet Jacobian terms of x on EVERY physical face: fface[f][c_t1 + fn1
// c_t2] = dt sum over the node's facets in face f of int g'(T_h) phi_I x_h ds,
// by the face workgroups of the marching launch (face_block: per facet, 3 x 3
// Gauss, four corners at once) over all six faces -- the marching tiles
// integrate the faces normal to their march axis themselves; the fused
// residual restriction (k_mg_rrestrict, tv_mg.hip) reads all six from here.
// (One thread per face node with facet_direct: 15.9 us at C4.)
template <int R>
__global__ __launch_bounds__(R * kWave) void k_cg_faces_all(CgGrid g, const double* __restrict__ T,
                                                            const double* __restrict__ x, FaceOff fo,
                                                            const PcgState* __restrict__ st) {
  if (st != nullptr && st->done) return;
  __shared__ double fsm[(8 * R + 8) * kWave];
  __shared__ double red[R];
  face_block<false, R>(g, T, x, x, x, 0.0, nullptr, RedTail{}, 0, (int)blockIdx.x, fo, fsm, red, 0);
}

}  // namespace

int launch_cg_japply_post(const CgGrid& g, const double* T, const double* x, const double* r, const double* dinv,
                          double omega, double* z, const PcgState* st, double* partials, const RedTail* tail,
                          hipStream_t s) {
  const Launch L = plan(g, false);
  // the production march configuration only; a partition's slab too (the march
  // writes z and its records on the owned planes only, the side-face pass skips
  // the ghost planes)
  if (!L.march || g.n0 < 3) return -1;
  const FaceOff fo = face_offsets(g, L.rows, 3 - L.raxis);
  const int grid = L.blocks + fo.off[6];
  const PostArgs pa{r, dinv, omega};
  hipLaunchKernelGGL((k_cg_march<MODE_JAC, false, 8, 1, 2, true>), dim3(grid), dim3(8 * kWave), 0, s, g, T, x,
                     nullptr, z, nullptr, st, partials, L.nseg, L.raxis, L.qchunk, RedTail{}, L.nparts, L.blocks, fo,
                     0, pa);
  const FaceAdd fa = cg_face_add(g, 0);
  const int nO = (L.raxis == 2) ? g.n1 : g.n2;
  const int64_t nodes = 2 * (int64_t)g.n1 * g.n2 + 2 * (int64_t)(g.n0 - 2) * nO;
  // 240 workgroups (some threads take two nodes): 11.6 -> 11.0 us at C4 against
  // one node per thread (319)
  constexpr int cap = 240;
  const int nb = (int)std::max<int64_t>(1, std::min<int64_t>((nodes + kBlock - 1) / kBlock, cap));
  const RedTail rt = tail ? *tail : RedTail{};
  hipLaunchKernelGGL(k_mg_post_faces, dim3(nb), dim3(kBlock), 0, s, fa, L.raxis, r, dinv, omega, z, partials,
                     L.blocks, rt, st, g.k_begin, g.k_end, g.w_begin, g.w_end);
  return L.blocks + nb;
}

bool cg_uses_march(const CgGrid& g) { return use_march(g); }

void launch_mg_prepare(const MgPrep& p, hipStream_t s) {
  const int64_t nn = p.off_n[p.nlev], nb = p.off_b[p.nlev];
  if (nn > 0) hipLaunchKernelGGL(k_mg_prep_inject, dim3((unsigned)((nn + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, p);
  if (nb > 0) hipLaunchKernelGGL(k_mg_prep_diag, dim3((unsigned)((nb + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, p);
}

int cg_num_blocks(const CgGrid& g, bool with_ghost_planes) { return plan(g, with_ghost_planes).nparts; }

FaceAdd cg_face_add(const CgGrid& g, int64_t t_off) {
  FaceAdd fa{};
  if (!use_march(g)) return fa;  // the row kernel keeps the facet terms inline
  fa.on = 1;
  fa.n0 = g.n0;
  fa.n1 = g.n1;
  fa.n2 = g.n2;
  fa.t_off = t_off;
  fa.inv_n0 = 1.0 / g.n0;
  fa.inv_plane = 1.0 / ((double)g.n0 * g.n1);
  const int qaxis = 3 - plan(g, true).raxis;  // faces normal to the march axis: added inside the march
  for (int f = 0; f < 6; ++f) fa.ff[f] = ((f >> 1) == qaxis) ? nullptr : g.fface[f];
  return fa;
}

void launch_cg_residual(const CgGrid& g, const double* T, const double* Tp, double* F, hipStream_t s) {
  launch_rows<MODE_RES, false>(g, T, T, Tp, F, nullptr, nullptr, nullptr, false, s);
}

bool launch_cg_residual_diag(const CgGrid& g, const double* T, const double* Tp, double* F, double* dinv,
                             hipStream_t s) {
  if (!use_march(g) || !g.bnodes || g.n_bnodes <= 0) return false;
  launch_rows<MODE_RES, false>(g, T, T, Tp, F, nullptr, nullptr, nullptr, false, s, nullptr, 0, true, dinv);
  return true;
}

void launch_cg_japply(const CgGrid& g, const double* T, const double* x, double* y, double* partials,
                      int* n_partials, hipStream_t s, const PcgState* st) {
  launch_rows<MODE_JAC, false>(g, T, x, nullptr, y, nullptr, st, partials, false, s);
  if (n_partials) *n_partials = plan(g, false).nparts;
}

bool launch_cg_japply_tail(const CgGrid& g, const double* T, const double* x, double* y, const PcgState* st,
                           double* partials, const RedTail* tail, hipStream_t s) {
  // complete J x (the face-workgroup terms added by k_cg_addfaces behind the
  // march) with the x.(J x) records of the march tiles and face workgroups
  // reduced by the tail into tail->out[0]
  return launch_rows<MODE_JAC, false>(g, T, x, nullptr, y, nullptr, st, partials, false, s, tail, 0, true);
}

void launch_cg_facet_faces(const CgGrid& g, const double* T, const double* x, const PcgState* st, hipStream_t s) {
  const FaceOff fo = face_offsets(g, kRows, -1);  // all six faces
  if (fo.off[6] <= 0) return;
  hipLaunchKernelGGL(k_cg_faces_all<kRows>, dim3(fo.off[6]), dim3(kRows * kWave), 0, s, g, T, x, fo, st);
}

// the six face arrays as a FaceAdd (every physical face, fface[] of g)
FaceAdd cg_face_add_all(const CgGrid& g) {
  FaceAdd fa = cg_face_add(g, 0);
  if (!fa.on) return fa;
  for (int f = 0; f < 6; ++f) fa.ff[f] = g.fface[f];
  return fa;
}

void launch_cg_japply_partial(const CgGrid& g, const double* T, const double* x, double* y, const PcgState* st,
                              hipStream_t s) {
  launch_rows<MODE_JAC, false>(g, T, x, nullptr, y, nullptr, st, nullptr, false, s, nullptr, 0, false);
}

bool launch_cg_japply_fused(const CgGrid& g, const double* T, const double* z, double* pA, double* pB,
                            double* w, const PcgState* st, double* partials, int* n_partials,
                            hipStream_t s, const RedTail* tail, int it_host) {
  // neighbour values of p_new are recomputed from z and p_old; p_new goes to the
  // other buffer of the pair (selected on device from st->it).
  // The march forms a lagged state with logic_update only (lag_update_lean):
  // any other lagged kind is refused (the callers then fail loudly)
  if (tail && tail->lag && tail->lag_kind != 3) return false;
  const bool fused = launch_rows<MODE_JAC, true>(g, T, z, pA, w, pB, st, partials, true, s, tail, it_host);
  if (n_partials) *n_partials = plan(g, true).nparts;
  return fused;
}

bool launch_cg_cgs(const CgGrid& g, bool init, const CgsBuffers& v, PcgState* st, double* partials,
                   hipStream_t s, const RedTail* tail, int it_host, const double* lag_sums) {
  if (!use_march(g)) return false;
  const Launch L = plan(g, true);
  const FaceOff fo = face_offsets(g, L.rows, 3 - L.raxis);
  const int grid = L.blocks + fo.off[6];
  RedTail rt{};
  if (tail) rt = *tail;
  if (init)
    hipLaunchKernelGGL((k_cgs_march<true, 8, 1>), dim3(grid), dim3(8 * kWave), 0, s, g, v, st, partials, L.nseg,
                       L.raxis, L.qchunk, rt, grid, L.blocks, fo, it_host, lag_sums);
  else
    hipLaunchKernelGGL((k_cgs_march<false, 8, 1>), dim3(grid), dim3(8 * kWave), 0, s, g, v, st, partials, L.nseg,
                       L.raxis, L.qchunk, rt, grid, L.blocks, fo, it_host, lag_sums);
  return true;
}

int cg_cgs_records(const CgGrid& g) {
  const Launch L = plan(g, true);
  return L.blocks + face_offsets(g, L.rows, 3 - L.raxis).off[6];
}

bool cg_cgs_supported(const CgGrid& g) { return use_march(g); }

void launch_cg_diag(const CgGrid& g, const double* T, double* dinv, int invert, hipStream_t s, bool bnd_only) {
  const int64_t nown = (int64_t)g.n0 * g.n1 * (g.w_end - g.w_begin);  // the write window
  int blocks = (int)std::min<int64_t>((nown + kBlock - 1) / kBlock, 4096);
  if (blocks <= 0) return;
  switch (dim_of(g)) {
    case 1: hipLaunchKernelGGL((k_cg_diag<1, true>), dim3(blocks), dim3(kBlock), 0, s, g, T, dinv, invert); break;
    case 2: hipLaunchKernelGGL((k_cg_diag<2, true>), dim3(blocks), dim3(kBlock), 0, s, g, T, dinv, invert); break;
    default:
      if (use_march(g) && g.bnodes && g.n_bnodes > 0) {  // the boundary-node list of the marching path
        // off the boundary diag J = diag(M + dt alpha K) does not depend on T:
        // bnd_only (the interior of dinv is already in place) rewrites the boundary nodes only
        if (!bnd_only) hipLaunchKernelGGL((k_cg_diag<3, false>), dim3(blocks), dim3(kBlock), 0, s, g, T, dinv, invert);
        hipLaunchKernelGGL(k_cg_diag_bnd, dim3(bnd_blocks(g)), dim3(kBlock), 0, s, g, T, dinv, invert);
      } else {
        hipLaunchKernelGGL((k_cg_diag<3, true>), dim3(blocks), dim3(kBlock), 0, s, g, T, dinv, invert);
      }
  }
}

}  // namespace tv
