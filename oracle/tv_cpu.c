/*
 * CPU ORACLE (C / OpenMP port) — test infrastructure only.
 *
 * A C restatement of the reference time step of pzimbrod/fem-glass-tempering
 * for structured 3D CG1 hexahedral plates (rectilinear grids), used as the
 * timed CPU baseline of bench.py ("kind": "port") and as a second CPU check.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
 * it; the product path never links it.
 *
 * Restates (file:line under /root/reference):
 *   residual F and Jacobian of ThermoViscoProblem.py:293-306 (CG branch),
 *   dolfinx NewtonSolver "incremental" (ThermoViscoProblem.py:334-337),
 *   PETSc KSPCG (:343) with a Jacobi preconditioner in place of GAMG (:344),
 *   the viscoelastic expressions ViscoelasticModel.py:100-228 in the call order
 *   of ThermoViscoProblem.py:393-595 (state fields only).
 * GMG (tvcpu_set_gmg): the geometric-multigrid preconditioner of the GPU's
 * bench line (fem-glass-tempering_amd/csrc/tv_mgsolve.cpp restated: the box
 * coarsened by two along every axis with >= 2 cells, plus the last node of an
 * odd count, until dt alpha / h^2 <= 0.5; re-discretised coarse operators with
 * T injected; damped Jacobi omega = 2 / (1.1 b), b the Gershgorin bound of
 * D^-1 J; one V-cycle with the same step before and after the coarse
 * correction, one Jacobi step on the coarsest level), in place of PETSc's
 * GAMG (ThermoViscoProblem.py:344) as on the GPU.
 * DG1 (tvcpu_create_dg): the SIPG residual / Jacobian of
 * ThermoViscoProblem.py:308-325 on the same rectilinear plates (cell-local
 * dofs, '+' = the lower cell, h = the '+' cell's diameter, penalty 5), the
 * same Newton / Jacobi-PCG / visco code on the 8 dofs of every cell.
 * Parity: unpinned against dolfinx (see oracle/tv_oracle.py); checked against
 * the numpy oracle in tests/test_cpu_port.py.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

enum { MLO, MDI, MUP, KLO, KDI, KUP, HLO, HHI, NC };

typedef struct {
  int n[3];
  long long N;
  double* c[3];
  double dt, dta, dtf, arad, aconv, Ta, Ta4;
  /* visco constants */
  double HoR, iTb, as_, dal;
  double lm[6], mn[6], lg[6], gn[6], lk[6], kn[6];
  /* state */
  double *T, *Tp, *Tf, *Tfp, *phi, *xi, *st, *sg, *sig;
  /* work */
  double *r, *z, *p, *w, *dx, *dinv;
  int last_newton, last_krylov;
  /* DG1: cell counts, cell lengths per axis; dof (l, cell) at l * ncell + cell */
  int dg, nc[3];
  long long ncell;
  double* hc[3];
  /* GMG (CG1): levels 1 .. nlev - 1 (level 0 = this grid) */
  int nlev;
  struct mglev* lev;
  double omega0, *x0;
} tvcpu;

/* one coarse level: its grid (the same operator code on its own tvcpu view),
 * vectors, weight and the transfer from the level above (per axis: 2
 * (index, weight) pairs per fine node, 3 per coarse node) */
typedef struct mglev {
  tvcpu g;                 /* n, c, N, T, dinv and the thermal constants of this level */
  double *b, *x, *w, omega;
  int *pi[3], *ri[3];
  double *pw[3], *rw[3];
  int fn[3];               /* node counts of the finer level */
} mglev;

static const double GX[3] = {0.11270166537925831148, 0.5, 0.88729833462074168852};
static const double GW[3] = {5.0 / 18.0, 8.0 / 18.0, 5.0 / 18.0};

static double gfun(const tvcpu* h, double T) {
  double T2 = T * T;
  return h->arad * (T2 * T2 - h->Ta4) + h->aconv * (T - h->Ta);
}
static double dgfun(const tvcpu* h, double T) { return h->arad * 4.0 * (T * T * T) + h->aconv; }

static void coefs(const double* X, int n, double* out) {
  for (int i = 0; i < n; ++i) {
    double* c = out + (size_t)i * NC;
    double hlo = i > 0 ? X[i] - X[i - 1] : 0.0, hhi = i < n - 1 ? X[i + 1] - X[i] : 0.0;
    c[MLO] = hlo / 6.0; c[MDI] = hlo / 3.0 + hhi / 3.0; c[MUP] = hhi / 6.0;
    c[KLO] = hlo > 0 ? -1.0 / hlo : 0.0;
    c[KDI] = (hlo > 0 ? 1.0 / hlo : 0.0) + (hhi > 0 ? 1.0 / hhi : 0.0);
    c[KUP] = hhi > 0 ? -1.0 / hhi : 0.0;
    c[HLO] = hlo; c[HHI] = hhi;
  }
}

/* facet integral around a boundary node; patches indexed [u+1][v+1] over the
 * face's two tangential axes. mode 0: g(T) phi ; 1: g'(T) phi p ; 2: g'(T) phi^2 */
static double facet(const tvcpu* h, int mode, const double* c1, const double* c2, double Tp[3][3], double Pp[3][3]) {
  double acc = 0.0;
  for (int s1 = 0; s1 < 2; ++s1) {
    double h1 = s1 ? c1[HHI] : c1[HLO];
    if (!(h1 > 0)) continue;
    int o1 = s1 ? 1 : -1;
    for (int s2 = 0; s2 < 2; ++s2) {
      double h2 = s2 ? c2[HHI] : c2[HLO];
      if (!(h2 > 0)) continue;
      int o2 = s2 ? 1 : -1;
      for (int q1 = 0; q1 < 3; ++q1) {
        double pc1 = s1 ? 1.0 - GX[q1] : GX[q1], po1 = 1.0 - pc1;
        for (int q2 = 0; q2 < 3; ++q2) {
          double pc2 = s2 ? 1.0 - GX[q2] : GX[q2], po2 = 1.0 - pc2;
          double w = GW[q1] * h1 * GW[q2] * h2, phi = pc1 * pc2;
          double Th = phi * Tp[1][1] + po1 * pc2 * Tp[1 + o1][1] + pc1 * po2 * Tp[1][1 + o2] + po1 * po2 * Tp[1 + o1][1 + o2];
          if (mode == 0) acc += w * gfun(h, Th) * phi;
          else if (mode == 2) acc += w * dgfun(h, Th) * phi * phi;
          else {
            double Ph = phi * Pp[1][1] + po1 * pc2 * Pp[1 + o1][1] + pc1 * po2 * Pp[1][1 + o2] + po1 * po2 * Pp[1 + o1][1 + o2];
            acc += w * dgfun(h, Th) * phi * Ph;
          }
        }
      }
    }
  }
  return h->dt * acc;
}

#define IDX(i, j, k) ((long long)(i) + (long long)n0 * ((j) + (long long)n1 * (k)))

static double at(const double* v, int n0, int n1, int n2, int i, int j, int k) {
  if (i < 0 || j < 0 || k < 0 || i >= n0 || j >= n1 || k >= n2) return 0.0;
  return v[IDX(i, j, k)];
}

/* mode 0: y = F(T; Tp) ; mode 1: y = J(T) x */
static void apply(tvcpu* h, int mode, const double* x, double* y) {
  const int n0 = h->n[0], n1 = h->n[1], n2 = h->n[2];
  const double* T = h->T;
  const double* Tp = h->Tp;
#pragma omp parallel for collapse(2) schedule(static)
  for (int k = 0; k < n2; ++k)
    for (int j = 0; j < n1; ++j) {
      const double *cy = h->c[1] + (size_t)j * NC, *cz = h->c[2] + (size_t)k * NC;
      for (int i = 0; i < n0; ++i) {
        const double* cx = h->c[0] + (size_t)i * NC;
        double S1[3], S2[3];
        for (int a = -1; a <= 1; ++a) {
          double s1 = 0.0, s2 = 0.0;
          for (int c = -1; c <= 1; ++c) {
            double us = 0.0, vs = 0.0, um = 0.0;
            for (int b = -1; b <= 1; ++b) {
              double xs = mode == 0 ? at(T, n0, n1, n2, i + a, j + b, k + c) : at(x, n0, n1, n2, i + a, j + b, k + c);
              us += cy[MDI + b] * xs;
              vs += cy[KDI + b] * xs;
              if (mode == 0) {
                int ok = !(i + a < 0 || j + b < 0 || k + c < 0 || i + a >= n0 || j + b >= n1 || k + c >= n2);
                double m = ok ? xs - at(Tp, n0, n1, n2, i + a, j + b, k + c) - h->dtf : 0.0;
                um += cy[MDI + b] * m;
              }
            }
            if (mode != 0) um = us;
            s1 += cz[MDI + c] * (um + h->dta * vs) + h->dta * cz[KDI + c] * us;
            s2 += cz[MDI + c] * us;
          }
          S1[a + 1] = s1;
          S2[a + 1] = h->dta * s2;
        }
        double v = 0.0;
        for (int a = -1; a <= 1; ++a) v += cx[MDI + a] * S1[a + 1] + cx[KDI + a] * S2[a + 1];
        /* facets */
        double Tpch[3][3], Ppch[3][3];
        const double* src = mode == 0 ? T : x;
        if (k == 0 || k == n2 - 1) {
          for (int u = 0; u < 3; ++u)
            for (int w = 0; w < 3; ++w) {
              Tpch[u][w] = at(T, n0, n1, n2, i + u - 1, j + w - 1, k);
              Ppch[u][w] = at(src, n0, n1, n2, i + u - 1, j + w - 1, k);
            }
          v += facet(h, mode == 0 ? 0 : 1, cx, cy, Tpch, Ppch);
        }
        if (j == 0 || j == n1 - 1) {
          for (int u = 0; u < 3; ++u)
            for (int w = 0; w < 3; ++w) {
              Tpch[u][w] = at(T, n0, n1, n2, i + u - 1, j, k + w - 1);
              Ppch[u][w] = at(src, n0, n1, n2, i + u - 1, j, k + w - 1);
            }
          v += facet(h, mode == 0 ? 0 : 1, cx, cz, Tpch, Ppch);
        }
        if (i == 0 || i == n0 - 1) {
          for (int u = 0; u < 3; ++u)
            for (int w = 0; w < 3; ++w) {
              Tpch[u][w] = at(T, n0, n1, n2, i, j + u - 1, k + w - 1);
              Ppch[u][w] = at(src, n0, n1, n2, i, j + u - 1, k + w - 1);
            }
          v += facet(h, mode == 0 ? 0 : 1, cy, cz, Tpch, Ppch);
        }
        y[IDX(i, j, k)] = v;
      }
    }
}

static void diag_inv(tvcpu* h) {
  const int n0 = h->n[0], n1 = h->n[1], n2 = h->n[2];
  const double* T = h->T;
#pragma omp parallel for collapse(2) schedule(static)
  for (int k = 0; k < n2; ++k)
    for (int j = 0; j < n1; ++j)
      for (int i = 0; i < n0; ++i) {
        const double *cx = h->c[0] + (size_t)i * NC, *cy = h->c[1] + (size_t)j * NC, *cz = h->c[2] + (size_t)k * NC;
        double d = cx[MDI] * cy[MDI] * cz[MDI] +
                   h->dta * (cx[KDI] * cy[MDI] * cz[MDI] + cx[MDI] * cy[KDI] * cz[MDI] + cx[MDI] * cy[MDI] * cz[KDI]);
        double P[3][3];
        if (k == 0 || k == n2 - 1) {
          for (int u = 0; u < 3; ++u) for (int w = 0; w < 3; ++w) P[u][w] = at(T, n0, n1, n2, i + u - 1, j + w - 1, k);
          d += facet(h, 2, cx, cy, P, P);
        }
        if (j == 0 || j == n1 - 1) {
          for (int u = 0; u < 3; ++u) for (int w = 0; w < 3; ++w) P[u][w] = at(T, n0, n1, n2, i + u - 1, j, k + w - 1);
          d += facet(h, 2, cx, cz, P, P);
        }
        if (i == 0 || i == n0 - 1) {
          for (int u = 0; u < 3; ++u) for (int w = 0; w < 3; ++w) P[u][w] = at(T, n0, n1, n2, i, j + u - 1, k + w - 1);
          d += facet(h, 2, cy, cz, P, P);
        }
        h->dinv[IDX(i, j, k)] = 1.0 / d;
      }
}

/* ---------------- DG1 (SIPG) ---------------- */
static double mloc(double hh, int a, int b) { return hh * (a == b ? (1.0 / 3.0) : (1.0 / 6.0)); }
static double kloc(double hh, int a, int b) { return (a == b ? 1.0 : -1.0) / hh; }

/* mode 0: y = F(T; Tp) ; 1: y = J(T) x ; 2: y = diag J(T) */
static void dg_apply(tvcpu* h, int mode, const double* x, double* y) {
  const int c0 = h->nc[0], c1 = h->nc[1], c2 = h->nc[2];
  const long long nce = h->ncell;
  const double* T = h->T;
  const long long cst[3] = {1, c0, (long long)c0 * c1};
  const int cn[3] = {c0, c1, c2};
  const double pen0 = 5.0;
#pragma omp parallel for schedule(static)
  for (long long cid = 0; cid < nce; ++cid) {
    const int ci[3] = {(int)(cid % c0), (int)((cid / c0) % c1), (int)(cid / ((long long)c0 * c1))};
    double hh[3], hd2 = 0.0;
    for (int k = 0; k < 3; ++k) {
      hh[k] = h->hc[k][ci[k]];
      hd2 += hh[k] * hh[k];
    }
    double u[8], m[8], yl[8];
    for (int l = 0; l < 8; ++l) {
      u[l] = mode == 0 ? T[l * nce + cid] : (mode == 1 ? x[l * nce + cid] : 0.0);
      m[l] = mode == 0 ? u[l] - h->Tp[l * nce + cid] - h->dtf : u[l];
    }
    /* cell term */
    for (int l = 0; l < 8; ++l) {
      double acc = 0.0;
      for (int q = 0; q < 8; ++q) {
        if (mode == 2 && q != l) continue;
        double mm = 1.0, kk = 0.0;
        for (int k = 0; k < 3; ++k) {
          const int a = (l >> k) & 1, b = (q >> k) & 1;
          double prod = kloc(hh[k], a, b);
          for (int e = 0; e < 3; ++e)
            if (e != k) prod *= mloc(hh[e], (l >> e) & 1, (q >> e) & 1);
          kk += prod;
          mm *= mloc(hh[k], a, b);
        }
        if (mode == 2) acc += mm + h->dta * kk;
        else acc += mm * m[q] + h->dta * kk * u[q];
      }
      yl[l] = acc;
    }
    /* facets */
    for (int k = 0; k < 3; ++k)
      for (int side = 0; side < 2; ++side) {
        const int nbi = ci[k] + (side ? 1 : -1);
        if (nbi >= 0 && nbi < cn[k]) {
          const long long nb = cid + (side ? cst[k] : -cst[k]);
          double un[8];
          for (int l = 0; l < 8; ++l) un[l] = mode == 0 ? T[l * nce + nb] : (mode == 1 ? x[l * nce + nb] : 0.0);
          const double hL = side ? hh[k] : h->hc[k][nbi], hR = side ? h->hc[k][nbi] : hh[k];
          const double pen = pen0 / sqrt(hd2 - hh[k] * hh[k] + hL * hL);
          const double Jv[4] = {0.0, 1.0, -1.0, 0.0};
          const double Gv[4] = {-0.5 / hL, 0.5 / hL, -0.5 / hR, 0.5 / hR};
          for (int l = 0; l < 8; ++l) {
            const int row = side ? ((l >> k) & 1) : 2 + ((l >> k) & 1);
            double acc = 0.0;
            for (int q = 0; q < 8; ++q) {
              if (mode == 2 && q != l) continue;
              const int bq = (q >> k) & 1;
              double mt = 1.0;
              for (int e = 0; e < 3; ++e)
                if (e != k) mt *= mloc(hh[e], (l >> e) & 1, (q >> e) & 1);
              const int co = side ? bq : 2 + bq, cb = side ? 2 + bq : bq;
              const double ao = pen * Jv[row] * Jv[co] - Gv[row] * Jv[co] - Jv[row] * Gv[co];
              const double an = pen * Jv[row] * Jv[cb] - Gv[row] * Jv[cb] - Jv[row] * Gv[cb];
              acc += mode == 2 ? mt * ao : mt * (ao * u[q] + an * un[q]);
            }
            yl[l] += h->dta * acc;
          }
        } else {
          /* Robin facet: 3 x 3 Gauss over the two tangential axes */
          double Tl[8];
          for (int l = 0; l < 8; ++l) Tl[l] = T[l * nce + cid];
          double acc[8] = {0};
          for (int qq = 0; qq < 9; ++qq) {
            double w = 1.0, xt[3] = {0.0, 0.0, 0.0};
            int t = 0;
            for (int e = 0; e < 3; ++e) {
              if (e == k) continue;
              const int qi = t == 0 ? qq % 3 : qq / 3;
              xt[e] = GX[qi];
              w *= GW[qi] * hh[e];
              ++t;
            }
            double phi[8], Th = 0.0, Ph = 0.0;
            for (int l = 0; l < 8; ++l) {
              double f = (((l >> k) & 1) == side) ? 1.0 : 0.0;
              for (int e = 0; e < 3; ++e)
                if (e != k) f *= ((l >> e) & 1) ? xt[e] : 1.0 - xt[e];
              phi[l] = f;
              Th += f * Tl[l];
              Ph += f * u[l];
            }
            for (int l = 0; l < 8; ++l) {
              if (mode == 0) acc[l] += w * gfun(h, Th) * phi[l];
              else if (mode == 1) acc[l] += w * dgfun(h, Th) * Ph * phi[l];
              else acc[l] += w * dgfun(h, Th) * phi[l] * phi[l];
            }
          }
          for (int l = 0; l < 8; ++l) yl[l] += h->dt * acc[l];
        }
      }
    for (int l = 0; l < 8; ++l) y[l * nce + cid] = yl[l];
  }
}

static void op_apply(tvcpu* h, int mode, const double* x, double* y) {
  if (h->dg) dg_apply(h, mode, x, y);
  else apply(h, mode, x, y);
}

static void op_diag_inv(tvcpu* h) {
  if (!h->dg) {
    diag_inv(h);
    return;
  }
  dg_apply(h, 2, NULL, h->dinv);
#pragma omp parallel for
  for (long long t = 0; t < h->N; ++t) h->dinv[t] = 1.0 / h->dinv[t];
}

/* ---------------- geometric multigrid (CG1) ---------------- */
static double gersh(const tvcpu* g) {
  /* max over nodes of the absolute row sum of M + dt alpha K over its diagonal
   * (= the max over the distinct per-axis row triples of the GPU's
   * mg_gershgorin); floor 2.25 for the Robin facet rows, then 5 % */
  double b = 0.0;
  const int n0 = g->n[0], n1 = g->n[1], n2 = g->n[2];
#pragma omp parallel for collapse(2) reduction(max : b)
  for (int k = 0; k < n2; ++k)
    for (int j = 0; j < n1; ++j)
      for (int i = 0; i < n0; ++i) {
        const double *r0 = g->c[0] + (size_t)i * NC, *r1 = g->c[1] + (size_t)j * NC, *r2 = g->c[2] + (size_t)k * NC;
        double sum = 0.0, diag = 0.0;
        for (int a = 0; a < 3; ++a)
          for (int bb = 0; bb < 3; ++bb)
            for (int cc = 0; cc < 3; ++cc) {
              double v = r0[a] * r1[bb] * r2[cc] +
                         g->dta * (r0[3 + a] * r1[bb] * r2[cc] + r0[a] * r1[3 + bb] * r2[cc] + r0[a] * r1[bb] * r2[3 + cc]);
              sum += fabs(v);
              if (a == 1 && bb == 1 && cc == 1) diag = v;
            }
        if (sum / diag > b) b = sum / diag;
      }
  return (b > 2.25 ? b : 2.25) * 1.05;
}

static void vcycle(tvcpu* h, int l, const double* b, double* x);

/* x_c(I) = fine value at the coarse node (injection, restriction entry 1) */
static void inject(const mglev* L, const double* Tf, double* Tc) {
  const int c0 = L->g.n[0], c1 = L->g.n[1], c2 = L->g.n[2], f0 = L->fn[0], f1 = L->fn[1];
#pragma omp parallel for collapse(2)
  for (int k = 0; k < c2; ++k)
    for (int j = 0; j < c1; ++j)
      for (int i = 0; i < c0; ++i)
        Tc[i + (long long)c0 * (j + (long long)c1 * k)] =
            Tf[L->ri[0][3 * i + 1] + (long long)f0 * (L->ri[1][3 * j + 1] + (long long)f1 * L->ri[2][3 * k + 1])];
}

/* bc = P^T (bf - wf) */
static void restrict_(const mglev* L, const double* bf, const double* wf, double* bc) {
  const int c0 = L->g.n[0], c1 = L->g.n[1], c2 = L->g.n[2], f0 = L->fn[0], f1 = L->fn[1];
#pragma omp parallel for collapse(2)
  for (int k = 0; k < c2; ++k)
    for (int j = 0; j < c1; ++j)
      for (int i = 0; i < c0; ++i) {
        double acc = 0.0;
        for (int c = 0; c < 3; ++c) {
          double pl = 0.0;
          for (int bb = 0; bb < 3; ++bb) {
            double row = 0.0;
            for (int a = 0; a < 3; ++a) {
              long long f = L->ri[0][3 * i + a] + (long long)f0 * (L->ri[1][3 * j + bb] + (long long)f1 * L->ri[2][3 * k + c]);
              row += L->rw[0][3 * i + a] * (bf[f] - wf[f]);
            }
            pl += L->rw[1][3 * j + bb] * row;
          }
          acc += L->rw[2][3 * k + c] * pl;
        }
        bc[i + (long long)c0 * (j + (long long)c1 * k)] = acc;
      }
}

/* xf += P xc */
static void prolong(const mglev* L, const double* xc, double* xf) {
  const int f0 = L->fn[0], f1 = L->fn[1], f2 = L->fn[2], c0 = L->g.n[0], c1 = L->g.n[1];
#pragma omp parallel for collapse(2)
  for (int k = 0; k < f2; ++k)
    for (int j = 0; j < f1; ++j)
      for (int i = 0; i < f0; ++i) {
        double acc = 0.0;
        for (int c = 0; c < 2; ++c)
          for (int bb = 0; bb < 2; ++bb)
            for (int a = 0; a < 2; ++a)
              acc += L->pw[2][2 * k + c] * L->pw[1][2 * j + bb] * L->pw[0][2 * i + a] *
                     xc[L->pi[0][2 * i + a] + (long long)c0 * (L->pi[1][2 * j + bb] + (long long)c1 * L->pi[2][2 * k + c])];
        xf[i + (long long)f0 * (j + (long long)f1 * k)] += acc;
      }
}

/* level l's grid, vectors and weight (level 0 = h itself) */
static tvcpu* lev_grid(tvcpu* h, int l) { return l == 0 ? h : &h->lev[l - 1].g; }
static double lev_omega(tvcpu* h, int l) { return l == 0 ? h->omega0 : h->lev[l - 1].omega; }
static double* lev_w(tvcpu* h, int l) { return l == 0 ? h->w : h->lev[l - 1].w; }

/* the V-cycle below level l: on entry x = omega D^-1 b (the pre-smoothing
 * step from 0); coarse correction; the same step after it */
static void vcycle(tvcpu* h, int l, const double* b, double* x) {
  if (l + 1 >= h->nlev) return;  /* coarsest: one Jacobi step */
  tvcpu* g = lev_grid(h, l);
  double* w = lev_w(h, l);
  mglev* C = &h->lev[l];
  apply(g, 1, x, w);
  restrict_(C, b, w, C->b);
  const long long Nc = C->g.N;
#pragma omp parallel for
  for (long long t = 0; t < Nc; ++t) C->x[t] = C->omega * C->g.dinv[t] * C->b[t];
  vcycle(h, l + 1, C->b, C->x);
  prolong(C, C->x, x);
  apply(g, 1, x, w);
  const double om = lev_omega(h, l);
  const long long N = g->N;
#pragma omp parallel for
  for (long long t = 0; t < N; ++t) x[t] += om * g->dinv[t] * (b[t] - w[t]);
}

/* z = B r: Jacobi, or one V-cycle (level 0 operands: h->x0 is the iterate) */
static void precond(tvcpu* h, const double* r, double* z) {
  const long long N = h->N;
  if (h->nlev <= 0) {
#pragma omp parallel for
    for (long long t = 0; t < N; ++t) z[t] = h->dinv[t] * r[t];
    return;
  }
#pragma omp parallel for
  for (long long t = 0; t < N; ++t) h->x0[t] = h->omega0 * h->dinv[t] * r[t];
  vcycle(h, 0, r, h->x0);
  memcpy(z, h->x0, sizeof(double) * (size_t)N);
}

/* per Newton iteration: T injected down the hierarchy, coarse diagonals */
static void mg_prepare(tvcpu* h) {
  const double* Tf = h->T;
  for (int l = 1; l < h->nlev; ++l) {
    mglev* L = &h->lev[l - 1];
    inject(L, Tf, L->g.T);
    diag_inv(&L->g);
    Tf = L->g.T;
  }
}

static void axis_tables(const double* Xf, int nf, const char* is_c, int* pi, double* pw, int* ri, double* rw) {
  int* cpos = (int*)malloc(sizeof(int) * nf);
  int* fpos = (int*)malloc(sizeof(int) * nf);
  int nc = 0;
  for (int i = 0; i < nf; ++i) {
    cpos[i] = -1;
    if (is_c[i]) { cpos[i] = nc; fpos[nc++] = i; }
  }
  for (int i = 0; i < nf; ++i) {
    if (is_c[i]) {
      pi[2 * i] = pi[2 * i + 1] = cpos[i];
      pw[2 * i] = 1.0;
      pw[2 * i + 1] = 0.0;
    } else {
      double wl = (Xf[i + 1] - Xf[i]) / (Xf[i + 1] - Xf[i - 1]);
      pi[2 * i] = cpos[i - 1];
      pi[2 * i + 1] = cpos[i + 1];
      pw[2 * i] = wl;
      pw[2 * i + 1] = 1.0 - wl;
    }
  }
  for (int I = 0; I < nc; ++I) {
    int fc = fpos[I];
    ri[3 * I] = ri[3 * I + 1] = ri[3 * I + 2] = fc;
    rw[3 * I] = rw[3 * I + 2] = 0.0;
    rw[3 * I + 1] = 1.0;
    if (fc - 1 >= 0 && !is_c[fc - 1]) { ri[3 * I] = fc - 1; rw[3 * I] = pw[2 * (fc - 1) + 1]; }
    if (fc + 1 < nf && !is_c[fc + 1]) { ri[3 * I + 2] = fc + 1; rw[3 * I + 2] = pw[2 * (fc + 1)]; }
  }
  free(cpos);
  free(fpos);
}

/* Deterministic dot products: fixed chunks of DCHUNK entries summed in order,
 * the chunk sums added in chunk order -- the same bits for any thread count
 * or schedule (OpenMP's reduction(+) combines the threads' partial sums in
 * arrival order, so Krylov counts at a convergence threshold could differ
 * between runs).  s2 / a2 may be NULL. */
#define DCHUNK 4096
static void dots(long long N, const double* a1, const double* b1, const double* a2, const double* b2, double* s1,
                 double* s2) {
  const long long nc = (N + DCHUNK - 1) / DCHUNK;
  double* part = (double*)malloc(sizeof(double) * 2 * (size_t)(nc > 0 ? nc : 1));
#pragma omp parallel for schedule(static)
  for (long long c = 0; c < nc; ++c) {
    const long long t1 = (c + 1) * DCHUNK < N ? (c + 1) * DCHUNK : N;
    double x = 0.0, y = 0.0;
    for (long long t = c * DCHUNK; t < t1; ++t) {
      x += a1[t] * b1[t];
      if (a2) y += a2[t] * b2[t];
    }
    part[2 * c] = x;
    part[2 * c + 1] = y;
  }
  double x = 0.0, y = 0.0;
  for (long long c = 0; c < nc; ++c) {
    x += part[2 * c];
    y += part[2 * c + 1];
  }
  free(part);
  *s1 = x;
  if (s2) *s2 = y;
}

static int pcg(tvcpu* h, double rtol) {
  const long long N = h->N;
  double zz = 0, zr = 0;
  if (h->nlev > 0) mg_prepare(h);
  precond(h, h->r, h->z);
#pragma omp parallel for
  for (long long t = 0; t < N; ++t) h->dx[t] = 0.0;
  dots(N, h->z, h->z, h->z, h->r, &zz, &zr);
  double dp = sqrt(zz), ttol = fmax(rtol * dp, 1e-50), rnorm0 = dp;
  if (dp <= ttol) return 0;
  double beta = zr, betaold = 1.0, dpiold = 0.0;
  for (int it = 0; it < 10000; ++it) {
    double b = it ? beta / betaold : 0.0;
#pragma omp parallel for
    for (long long t = 0; t < N; ++t) h->p[t] = it ? h->z[t] + b * h->p[t] : h->z[t];
    op_apply(h, 1, h->p, h->w);
    double dpi = 0;
    dots(N, h->p, h->w, NULL, NULL, &dpi, NULL);
    if (dpi == 0.0 || (it > 0 && (dpi > 0) != (dpiold > 0))) return -it - 1;
    dpiold = dpi;
    betaold = beta;
    double a = beta / dpi;
    zz = 0; zr = 0;
#pragma omp parallel for
    for (long long t = 0; t < N; ++t) {
      h->dx[t] += a * h->p[t];
      h->r[t] -= a * h->w[t];
    }
    precond(h, h->r, h->z);
    dots(N, h->z, h->z, h->z, h->r, &zz, &zr);
    dp = sqrt(zz);
    if (dp <= ttol) return it + 1;
    if (dp >= 1e5 * rnorm0 || !isfinite(dp)) return -it - 1;
    beta = zr;
  }
  return -10001;
}

static int newton(tvcpu* h) {
  const long long N = h->N;
  int its = 0, kits = 0, conv = 0;
  double r0 = 0.0;
  op_apply(h, 0, NULL, h->r);
  while (!conv && its < 50) {
    op_diag_inv(h);
    int k = pcg(h, 1e-5);
    if (k < 0) return -1;
    kits += k;
    double nn = 0;
#pragma omp parallel for
    for (long long t = 0; t < N; ++t) h->T[t] -= h->dx[t];
    dots(N, h->dx, h->dx, NULL, NULL, &nn, NULL);
    double rn = sqrt(nn);
    ++its;
    if (its == 1) r0 = rn;
    else conv = (rn / r0 < 1e-12) || (rn < 1e-10);
    if (!conv) op_apply(h, 0, NULL, h->r);
  }
  h->last_newton = its;
  h->last_krylov = kits;
  return conv ? 0 : -2;
}

static double tE(double xi, double lam) {
  double x = (-xi) / lam;
  return (1.0 + 1.0 * x) + 0.5 * (x * x);
}

static void visco(tvcpu* h) {
  const long long N = h->N;
#pragma omp parallel for schedule(static)
  for (long long t = 0; t < N; ++t) {
    double T = h->T[t], Tp = h->Tp[t];
    double phi = exp(h->HoR * (h->iTb - 1.0 / T));
    double Tf = 0.0;
    for (int i = 0; i < 6; ++i) {
      double cur = (h->lm[i] * h->Tfp[i * N + t] + T * h->dt * phi) / (h->lm[i] + h->dt * phi);
      h->Tfp[i * N + t] = cur;
      Tf = Tf + h->mn[i] * cur;
    }
    h->Tf[t] = Tf;
    double scal = h->as_ * (T - Tp) + h->dal * (Tf - Tf);
    double tot[9], dev[9], tr = 0.0;
    for (int q = 0; q < 9; ++q) tot[q] = -(((q / 3) == (q % 3) ? 1.0 : 0.0) * scal);
    for (int i = 0; i < 3; ++i) tr = tr + tot[4 * i];
    for (int q = 0; q < 9; ++q) dev[q] = tot[q] - ((1.0 / 3.0) * ((q / 3) == (q % 3) ? 1.0 : 0.0)) * tr;
    double Tn = T + (T - Tp);
    double phin = exp(h->HoR * (h->iTb - 1.0 / Tn));
    double xi = (h->dt / 2) * (phin - phi);
    h->phi[t] = phi;
    h->xi[t] = xi;
    double sig[9];
    for (int n = 0; n < 6; ++n) {
      double Eg = tE(xi, h->lg[n]), Ek = tE(xi, h->lk[n]);
      for (int q = 0; q < 9; ++q) {
        long long o = (long long)(n * 9 + q) * N + t;
        double ds = (((2.0 * h->gn[n] * dev[q]) / xi) * h->lg[n]) * (1.0 - Eg);
        double stv = h->st[o] * Eg;
        double dsg = (((h->kn[n] * (tr * ((q / 3) == (q % 3) ? 1.0 : 0.0))) / xi) * h->lk[n]) * (1.0 - Ek);
        double sgv = h->sg[o] * Ek;
        h->st[o] = stv;
        h->sg[o] = sgv;
        double add = (ds + stv) + (dsg + sgv);
        sig[q] = n == 0 ? add : sig[q] + add;
      }
    }
    for (int q = 0; q < 9; ++q) h->sig[(long long)q * N + t] = sig[q];
    h->Tp[t] = T;
  }
}

/* ---------------- C entry points (ctypes) ---------------- */
static void* create(int dg, const int* ncells, const double* x, const double* y, const double* z,
                    const double* params, const double* tabs) {
  tvcpu* h = (tvcpu*)calloc(1, sizeof(tvcpu));
  const double* X[3] = {x, y, z};
  h->dg = dg;
  for (int a = 0; a < 3; ++a) {
    h->n[a] = ncells[a] + 1;
    h->c[a] = (double*)malloc(sizeof(double) * NC * h->n[a]);
    coefs(X[a], h->n[a], h->c[a]);
    h->nc[a] = ncells[a];
    h->hc[a] = (double*)malloc(sizeof(double) * (size_t)ncells[a]);
    for (int i = 0; i < ncells[a]; ++i) h->hc[a][i] = X[a][i + 1] - X[a][i];
  }
  h->ncell = (long long)ncells[0] * ncells[1] * ncells[2];
  h->N = dg ? 8 * h->ncell : (long long)h->n[0] * h->n[1] * h->n[2];
  double f = params[0], eps = params[1], sg = params[2], Ta = params[3], T0 = params[4], al = params[5], htc = params[6];
  h->dt = params[12];
  h->dta = h->dt * al;
  h->dtf = h->dt * f;
  h->arad = 0.001 * (sg * eps);
  h->aconv = 0.001 * htc;
  h->Ta = Ta;
  h->Ta4 = Ta * Ta * Ta * Ta;
  h->HoR = params[7] / params[9];
  h->iTb = 1.0 / params[8];
  h->as_ = params[10];
  h->dal = params[11] - params[10];
  for (int i = 0; i < 6; ++i) {
    h->mn[i] = tabs[i]; h->lm[i] = tabs[6 + i]; h->gn[i] = tabs[12 + i];
    h->lg[i] = tabs[18 + i]; h->kn[i] = tabs[24 + i]; h->lk[i] = tabs[30 + i];
  }
  const long long N = h->N;
  double** bufs[] = {&h->T, &h->Tp, &h->Tf, &h->phi, &h->xi, &h->r, &h->z, &h->p, &h->w, &h->dx, &h->dinv};
  for (size_t q = 0; q < sizeof(bufs) / sizeof(bufs[0]); ++q) *bufs[q] = (double*)calloc((size_t)N, sizeof(double));
  h->Tfp = (double*)calloc((size_t)N * 6, sizeof(double));
  h->st = (double*)calloc((size_t)N * 54, sizeof(double));
  h->sg = (double*)calloc((size_t)N * 54, sizeof(double));
  h->sig = (double*)calloc((size_t)N * 9, sizeof(double));
#pragma omp parallel for
  for (long long t = 0; t < N; ++t) {
    h->T[t] = T0; h->Tp[t] = T0; h->Tf[t] = T0;
    for (int i = 0; i < 6; ++i) h->Tfp[i * N + t] = T0;
  }
  return h;
}

void* tvcpu_create(const int* ncells, const double* x, const double* y, const double* z,
                   const double* params /* f eps sigma Ta T0 alpha htc H Tb Rg as al dt */,
                   const double* tabs /* 36: m lm g lg k lk */) {
  return create(0, ncells, x, y, z, params, tabs);
}

/* DG1 temperature and stress spaces; dofs (l, cell) at l * ncell + cell with
 * l = bx + 2 by + 4 bz the cell corner */
void* tvcpu_create_dg(const int* ncells, const double* x, const double* y, const double* z, const double* params,
                      const double* tabs) {
  return create(1, ncells, x, y, z, params, tabs);
}

int tvcpu_step(void* hp, int thermal_only, int* newton_its, int* krylov_its) {
  tvcpu* h = (tvcpu*)hp;
  int rc = newton(h);
  if (rc) return rc;
  if (!thermal_only) visco(h);
  else memcpy(h->Tp, h->T, sizeof(double) * (size_t)h->N);
  if (newton_its) *newton_its = h->last_newton;
  if (krylov_its) *krylov_its = h->last_krylov;
  return 0;
}

long long tvcpu_num_dofs(void* hp) { return ((tvcpu*)hp)->N; }

/* switch the Krylov preconditioner of a CG1 plate to the geometric multigrid
 * (the hierarchy of tv_mgsolve.cpp mg_setup, automatic depth); returns the
 * number of levels incl. the fine one, or -1 (DG: not supported here) */
int tvcpu_set_gmg(void* hp) {
  tvcpu* h = (tvcpu*)hp;
  if (h->dg) return -1;
  const double da = h->dta;
  /* node coordinates of the current level, per axis */
  double* X[3];
  int n[3];
  for (int a = 0; a < 3; ++a) {
    n[a] = h->n[a];
    X[a] = (double*)malloc(sizeof(double) * n[a]);
    /* rebuild the coordinates from the cell lengths */
    X[a][0] = 0.0;
    for (int i = 1; i < n[a]; ++i) X[a][i] = X[a][i - 1] + h->c[a][(size_t)i * NC + HLO];
  }
  h->lev = (mglev*)calloc(16, sizeof(mglev));
  h->nlev = 1;
  h->omega0 = 2.0 / (1.1 * gersh(h));
  for (int lev = 1; lev < 8; ++lev) {
    double hmin = 1e300;
    int coarse[3], any = 0;
    for (int a = 0; a < 3; ++a) {
      int cells = n[a] - 1;
      coarse[a] = cells >= 2;
      any |= coarse[a];
      if (cells >= 1) {
        double m = (X[a][n[a] - 1] - X[a][0]) / cells;
        if (m < hmin) hmin = m;
      }
    }
    if (!any || da / (hmin * hmin) <= 0.5) break;
    mglev* L = &h->lev[lev - 1];
    double* Xc[3];
    int nc[3];
    for (int a = 0; a < 3; ++a) {
      char* is_c = (char*)malloc(n[a]);
      int m = 0;
      for (int i = 0; i < n[a]; ++i) {
        is_c[i] = coarse[a] ? ((i % 2 == 0 || i == n[a] - 1) ? 1 : 0) : 1;
        m += is_c[i];
      }
      nc[a] = m;
      Xc[a] = (double*)malloc(sizeof(double) * m);
      for (int i = 0, q = 0; i < n[a]; ++i)
        if (is_c[i]) Xc[a][q++] = X[a][i];
      L->pi[a] = (int*)malloc(sizeof(int) * 2 * n[a]);
      L->pw[a] = (double*)malloc(sizeof(double) * 2 * n[a]);
      L->ri[a] = (int*)malloc(sizeof(int) * 3 * m);
      L->rw[a] = (double*)malloc(sizeof(double) * 3 * m);
      axis_tables(X[a], n[a], is_c, L->pi[a], L->pw[a], L->ri[a], L->rw[a]);
      L->fn[a] = n[a];
      free(is_c);
    }
    /* the level's grid: the fine grid's constants, its own coefficients and vectors */
    tvcpu* g = &L->g;
    memcpy(g, h, sizeof(tvcpu));
    g->nlev = 0;
    g->lev = NULL;
    for (int a = 0; a < 3; ++a) {
      g->n[a] = nc[a];
      g->c[a] = (double*)malloc(sizeof(double) * NC * nc[a]);
      coefs(Xc[a], nc[a], g->c[a]);
    }
    g->N = (long long)nc[0] * nc[1] * nc[2];
    g->T = (double*)calloc((size_t)g->N, sizeof(double));
    g->dinv = (double*)calloc((size_t)g->N, sizeof(double));
    L->b = (double*)calloc((size_t)g->N, sizeof(double));
    L->x = (double*)calloc((size_t)g->N, sizeof(double));
    L->w = (double*)calloc((size_t)g->N, sizeof(double));
    L->omega = 2.0 / (1.1 * gersh(g));
    for (int a = 0; a < 3; ++a) {
      free(X[a]);
      X[a] = Xc[a];
      n[a] = nc[a];
    }
    h->nlev = lev + 1;
  }
  for (int a = 0; a < 3; ++a) free(X[a]);
  h->x0 = (double*)calloc((size_t)h->N, sizeof(double));
  return h->nlev;
}

/* z = B r with the current preconditioner at the current T (tests) */
void tvcpu_precond_apply(void* hp, const double* r, double* z) {
  tvcpu* h = (tvcpu*)hp;
  diag_inv(h);
  if (h->nlev > 0) mg_prepare(h);
  precond(h, r, z);
}

void tvcpu_get(void* hp, int which, double* out) {
  tvcpu* h = (tvcpu*)hp;
  const long long N = h->N;
  switch (which) {
    case 0: memcpy(out, h->T, sizeof(double) * N); break;
    case 1: memcpy(out, h->phi, sizeof(double) * N); break;
    case 2: memcpy(out, h->xi, sizeof(double) * N); break;
    case 3: memcpy(out, h->Tf, sizeof(double) * N); break;
    case 4: /* sigma, interleaved dof*9+q */
      for (long long t = 0; t < N; ++t)
        for (int q = 0; q < 9; ++q) out[t * 9 + q] = h->sig[(long long)q * N + t];
      break;
  }
}

int tvcpu_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

void tvcpu_destroy(void* hp) {
  tvcpu* h = (tvcpu*)hp;
  if (!h) return;
  double* bufs[] = {h->T, h->Tp, h->Tf, h->phi, h->xi, h->r, h->z, h->p, h->w, h->dx, h->dinv, h->Tfp, h->st, h->sg, h->sig,
                    h->c[0], h->c[1], h->c[2], h->hc[0], h->hc[1], h->hc[2]};
  for (size_t q = 0; q < sizeof(bufs) / sizeof(bufs[0]); ++q) free(bufs[q]);
  for (int l = 1; l < h->nlev; ++l) {
    mglev* L = &h->lev[l - 1];
    double* lb[] = {L->b, L->x, L->w, L->g.T, L->g.dinv, L->g.c[0], L->g.c[1], L->g.c[2],
                    L->pw[0], L->pw[1], L->pw[2], L->rw[0], L->rw[1], L->rw[2]};
    for (size_t q = 0; q < sizeof(lb) / sizeof(lb[0]); ++q) free(lb[q]);
    for (int a = 0; a < 3; ++a) { free(L->pi[a]); free(L->ri[a]); }
  }
  free(h->lev);
  free(h->x0);
  free(h);
}
