// Host runtime of libtvfem.so: context, mesh partition, device state, field
// transfer, the Newton + Jacobi-PCG driver, the viscoelastic step and the RCCL
// halo / reductions.  C-ABI in include/tvfem.h.
//
// Reference mapping (file:line under /root/reference):
//   Ctx construction      ThermoViscoProblem.__init__ (ThermoViscoProblem.py:24-58)
//   initial condition     _set_initial_condition (:187-233)
//   tv_solve_T            _solve_T (:384-391) -> dolfinx NewtonSolver [3P]
//                         configured at _setup_solver (:330-346)
//   tv_visco_update       _solve_Tf .. _solve_stress (:393-595)
//   tv_step               solve_timestep (:367-381) without _write_output
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "tv_internal.h"

namespace tv {

static std::mutex g_err_mu;
static std::string g_err;

static void set_global_error(const std::string& m) {
  std::lock_guard<std::mutex> lk(g_err_mu);
  g_err = m;
}

const char* experiment_env(const char* name) {
  static std::mutex mu;
  static std::vector<std::string> reported;
  const char* gate = getenv("TVFEM_EXPERIMENTS");
  if (!gate || std::strcmp(gate, "1") != 0) return nullptr;
  const char* v = getenv(name);
  if (!v) return nullptr;
  std::lock_guard<std::mutex> lk(mu);
  if (std::find(reported.begin(), reported.end(), name) == reported.end()) {
    reported.emplace_back(name);
    std::fprintf(stderr, "[tvfem] experiment switch %s=%s active (TVFEM_EXPERIMENTS=1)\n", name, v);
  }
  return v;
}

struct FieldInfo {
  double* ptr = nullptr;
  int bs = 1;       // components
  int space = 0;    // 0 T space, 1 sigma space
  bool alloc = false;
};

// One coarse level of the geometric-multigrid hierarchy (tv_mg.hip): a
// single-partition CG grid of the box coarsened by two along the axes with an
// even cell count, its transfer from the next finer level and its vectors.
struct MgLevel {
  CgGrid g{};
  std::vector<double> X[3];  // storage-axis node coordinates
  int64_t n = 0;
  double omega = 0.0;        // damped-Jacobi weight 2 / (1.1 b), b >= lambda_max(D^-1 J)
  double *T = nullptr, *b = nullptr, *x = nullptr, *w = nullptr, *dinv = nullptr;
  MgXfer xf{};               // finer level -> this level
  double* coef[3] = {nullptr, nullptr, nullptr};
  int64_t* bnodes = nullptr;
  double* ffbuf[2] = {nullptr, nullptr};
  std::vector<void*> bufs;   // T, b, x, w, dinv and the transfer maps
  bool dinv_interior = false;  // dinv holds the T-independent interior diagonal
};

struct Ctx {
  std::string err;
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  hipEvent_t evp[2] = {nullptr, nullptr};  // PCG convergence polls (double-buffered)
  tv_params P{};
  tv_options O{};
  int dim = 1;
  int fam_T = TV_CG, fam_S = TV_CG;
  int perm[3] = {0, -1, -1};  // storage axis -> physical axis (-1 degenerate)
  int n_parts = 1, part = 0;
  // global / local sizes
  int Nnode_glob[3] = {1, 1, 1};  // per storage axis
  int Ncell_glob[3] = {0, 0, 0};
  int plane_begin = 0, plane_end = 0;  // owned global planes (CG) / cell layers (DG) along storage axis 2
  CgGrid cg{};
  bool dinv_interior = false;  // dinv holds the T-independent interior diagonal (CG march path)
  DgGrid dg{};
  int64_t nT = 0, nS = 0;          // local dofs incl. ghosts
  int64_t ownT_off = 0, ownT_n = 0;
  int64_t ownS_off = 0, ownS_n = 0;
  int64_t globT_off = 0, globS_off = 0;
  std::vector<std::vector<double>> coords;  // physical axes
  FieldInfo f[TV_NUM_FIELDS];
  double* coef[3] = {nullptr, nullptr, nullptr};
  double* dgh[3] = {nullptr, nullptr, nullptr};
  int* map = nullptr;
  int64_t* bnodes = nullptr;
  double* ffbuf[2] = {nullptr, nullptr};  // Robin facet-term face arrays (CgGrid::ffbuf)
  // PCG work (T space, local size)
  double *r = nullptr, *z = nullptr, *pA = nullptr, *pB = nullptr, *w = nullptr, *dinv = nullptr;
  // single-reduction PCG (k_cgs_march): r, s, w in two parities (w[0] = w);
  // p = pA, x = the dx field; wsend: the two packed boundary planes of w + facet
  // terms sent to the neighbours (multi-rank)
  bool cgs = false;
  // Dirichlet mode (tv_set_dirichlet): dB = T - value on the boundary nodes, tmp = J dB
  bool dir_on = false;
  double dir_value = 0.0;
  double *dB = nullptr, *dtmp = nullptr;
  double* Tfo = nullptr;  // paper mode, mixed families: previous Tf per T dof
  Output* out = nullptr;  // time-series output (tv_output_*)
  // geometric multigrid (options.preconditioner = TV_PC_GMG): levels 1.. (level 0 = cg)
  bool mg_on = false;
  bool mg_dg = false;       // DG1 level 0 over the CG1 hierarchy of the same box
  std::vector<MgLevel> mg;
  double mg_omega0 = 0.0;
  double* mgx = nullptr;    // level-0 V-cycle iterate
  double* dggface = nullptr; // DG level 0: facet means of dg(T) for the cell-block Jacobi smoother
  // unstructured mesh (tv_create_unstructured, tv_um.hip)
  bool um = false;
  UmGrid umg{};
  std::vector<double> um_xyz;        // host copy: 3 per vertex
  std::vector<int64_t> um_cells;     // host copy: 2^dim per cell (input order)
  UmDevice* umd = nullptr;            // assembled operators, facet data (tv_um.hip)
  unsigned char* um_bmask = nullptr;  // boundary vertices (Dirichlet mode)
  std::vector<int> out_fields;
  double *cr[2] = {nullptr, nullptr}, *cs[2] = {nullptr, nullptr}, *cw1 = nullptr;
  double* wsend = nullptr;
  double* partials = nullptr;
  int n_partials_cap = 0;
  double* sums = nullptr;
  unsigned* counters = nullptr;  // arrival counters of the in-kernel reduction tails
  PcgState* st = nullptr;
  PcgState* h_st = nullptr;  // pinned, 3 slots: 0 / 1 the PCG polls, 2 the state uploaded at a solve's start
  double* h_sums = nullptr;  // pinned
  int* tflag = nullptr;       // device: s_tilde / sigma_tilde all +0.0 (0) or general (1), see ViscoFields
  double* scratch = nullptr;  // transfer scratch
  size_t scratch_bytes = 0;
  // comm: RCCL (production) or host-staged callbacks (testing several ranks on one GPU)
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0;
  tv_host_allreduce_fn host_allreduce = nullptr;
  tv_host_sendrecv_fn host_sendrecv = nullptr;
  void* host_user = nullptr;
  double* h_halo = nullptr;  // pinned staging: 2 send + 2 recv planes
  size_t h_halo_n = 0;
  // in-solve kernel timing (tv_kernel_timing): the fused matvec and the PCG
  // update stamp the device REALTIME clock at their start (workgroup 0) and at
  // the end of their reduction tail into d_ts (4 stamps per PCG iteration, one
  // slot per iteration, read back in bulk); HIP events around the visco update
  bool ktime = false;
  int kstride = 1;                   // every kstride-th PCG iteration is timed
  uint64_t* d_ts = nullptr;          // kTsCap slots x {matvec start, end, update start, end}
  int ts_next = 0;                   // first free slot
  std::vector<int> ts_pending;       // slots of productive iterations not yet read back
  double ts_khz = 0.0;               // REALTIME clock (hipDeviceAttributeWallClockRate)
  hipEvent_t vev[2] = {nullptr, nullptr};
  double ksum[3] = {0.0, 0.0, 0.0};  // ms: fused matvec, PCG update, visco update
  int64_t kcnt[3] = {0, 0, 0};
  // stats
  int last_newton = 0, last_krylov = 0;
  double last_dx = 0.0;
  int pcg_hint = 0;

  int fail(int code, const std::string& m) {
    err = m;
    return code;
  }
};

#define HIPC(expr)                                                                              \
  do {                                                                                          \
    hipError_t e_ = (expr);                                                                     \
    if (e_ != hipSuccess)                                                                       \
      return c->fail(TV_ERR_HIP, std::string("HIP error ") + hipGetErrorString(e_) + " at " +  \
                                     __FILE__ + ":" + std::to_string(__LINE__) + ": " #expr); \
  } while (0)

#define NCCLC(expr)                                                                             \
  do {                                                                                          \
    ncclResult_t r_ = (expr);                                                                   \
    if (r_ != ncclSuccess)                                                                      \
      return c->fail(TV_ERR_COMM, std::string("RCCL error ") + ncclGetErrorString(r_) + " at " + \
                                      std::to_string(__LINE__) + ": " #expr);                   \
  } while (0)

// --------------------------------------------------------------------------------------
// geometry helpers
// --------------------------------------------------------------------------------------
static void axis_coefs(const std::vector<double>& X, int first, int count, std::vector<double>& out) {
  // 1D P1 assembled mass / stiffness rows and adjacent cell lengths for global
  // nodes [first, first+count) of an axis with node coordinates X.
  const int n = (int)X.size();
  out.assign((size_t)count * C_NCOEF, 0.0);
  for (int q = 0; q < count; ++q) {
    const int i = first + q;
    double* c = &out[(size_t)q * C_NCOEF];
    if (n == 1) {
      c[C_MDI] = 1.0;
      continue;
    }
    const double hlo = (i > 0) ? X[i] - X[i - 1] : 0.0;
    const double hhi = (i < n - 1) ? X[i + 1] - X[i] : 0.0;
    c[C_MLO] = hlo / 6.0;
    c[C_MDI] = hlo / 3.0 + hhi / 3.0;
    c[C_MUP] = hhi / 6.0;
    c[C_KLO] = hlo > 0 ? -1.0 / hlo : 0.0;
    c[C_KDI] = (hlo > 0 ? 1.0 / hlo : 0.0) + (hhi > 0 ? 1.0 / hhi : 0.0);
    c[C_KUP] = hhi > 0 ? -1.0 / hhi : 0.0;
    c[C_HLO] = hlo;
    c[C_HHI] = hhi;
  }
}

static const std::vector<double>& storage_coords(Ctx* c, int s, std::vector<double>& tmp) {
  if (c->perm[s] < 0) {
    tmp.assign(1, 0.0);
    return tmp;
  }
  return c->coords[c->perm[s]];
}

static int alloc_field(Ctx* c, int id, int space, int bs) {
  FieldInfo& fi = c->f[id];
  fi.space = space;
  fi.bs = bs;
  const int64_t n = (space == 0 ? c->nT : c->nS);
  HIPC(hipMalloc(&fi.ptr, sizeof(double) * (size_t)std::max<int64_t>(1, n * bs)));
  HIPC(hipMemsetAsync(fi.ptr, 0, sizeof(double) * (size_t)(n * bs), c->stream));
  fi.alloc = true;
  return TV_OK;
}

static void alias_field(Ctx* c, int id, int target) {
  c->f[id] = c->f[target];
  c->f[id].alloc = false;
}

// storage axes: 0 = x (fastest); 2 = partition axis (slowest); 1 = the remaining
// axis (or degenerate).  Returns false for an invalid part_axis.
static bool storage_perm(const tv_mesh_desc* m, int perm[3]) {
  const int d = m->dim;
  if (d == 1) {
    perm[0] = 0; perm[1] = -1; perm[2] = -1;
  } else if (d == 2) {
    perm[0] = 0; perm[1] = -1; perm[2] = 1;
  } else {
    int pa = m->part_axis;
    if (pa < 0) pa = (m->n_cells[1] >= m->n_cells[2]) ? 1 : 2;
    if (pa != 1 && pa != 2) return false;
    perm[0] = 0; perm[2] = pa; perm[1] = (pa == 1) ? 2 : 1;
  }
  return true;
}

// owned node planes [b0, b1) of partition p of P along the slowest storage axis
static void part_planes(int N2, int P, int p, int* b0, int* b1) {
  *b0 = (int)((int64_t)N2 * p / P);
  *b1 = (int)((int64_t)N2 * (p + 1) / P);
}

// CG grid of `n2` local planes starting at global plane `first2` of storage
// axis 2 (ghost planes included: g_lo / g_hi of them), from the global node
// coordinates X[s] of the storage axes (a single 0 for a degenerate axis);
// bnd2lo / bnd2hi: the low / high face of axis 2 is a physical boundary here.
// Device arrays go to coef[3], *bnodes and ffbuf[2] (owned by the caller).
static int build_cg_grid(Ctx* c, int d, const std::vector<double> (&X)[3], int first2, int n2, int g_lo, int g_hi,
                         bool bnd2lo, bool bnd2hi, CgGrid& g, double** coef, int64_t** bnodes, double** ffbuf) {
  g.n0 = (int)X[0].size();
  g.n1 = (int)X[1].size();
  g.g_lo = g_lo;
  g.g_hi = g_hi;
  g.n2 = n2;
  g.k_begin = g_lo;
  g.k_end = n2 - g_hi;
  g.deg1 = X[1].size() == 1;
  g.deg2 = X[2].size() == 1;
  g.bnd[0][0] = g.bnd[0][1] = 1;
  g.bnd[1][0] = g.bnd[1][1] = g.deg1 ? 0 : 1;
  g.bnd[2][0] = (!g.deg2 && bnd2lo) ? 1 : 0;
  g.bnd[2][1] = (!g.deg2 && bnd2hi) ? 1 : 0;
  const int first[3] = {0, 0, first2};
  const int cnt[3] = {g.n0, g.n1, g.n2};
  for (int s = 0; s < 3; ++s) {
    std::vector<double> cf;
    axis_coefs(X[s], first[s], cnt[s], cf);
    HIPC(hipMalloc(&coef[s], cf.size() * sizeof(double)));
    HIPC(hipMemcpy(coef[s], cf.data(), cf.size() * sizeof(double), hipMemcpyHostToDevice));
    g.coef[s] = coef[s];
  }
  const int64_t plane = (int64_t)g.n0 * g.n1;
  for (int f = 0; f < 6; ++f) g.ffoff[f] = -1;
  if (d == 3) {  // owned nodes on physical boundary faces (Robin facets, marching kernel path)
    std::vector<int64_t> bn;
    for (int k = g.k_begin; k < g.k_end; ++k)
      for (int j = 0; j < g.n1; ++j)
        for (int i = 0; i < g.n0; ++i) {
          const bool on = (i == 0 && g.bnd[0][0]) || (i == g.n0 - 1 && g.bnd[0][1]) ||
                          (j == 0 && g.bnd[1][0]) || (j == g.n1 - 1 && g.bnd[1][1]) ||
                          (k == 0 && g.bnd[2][0]) || (k == g.n2 - 1 && g.bnd[2][1]);
          if (on) bn.push_back((int64_t)i + (int64_t)g.n0 * j + plane * k);
        }
    if (!bn.empty()) {
      HIPC(hipMalloc(bnodes, bn.size() * sizeof(int64_t)));
      HIPC(hipMemcpy(*bnodes, bn.data(), bn.size() * sizeof(int64_t), hipMemcpyHostToDevice));
    }
    g.bnodes = *bnodes;
    g.n_bnodes = (int64_t)bn.size();
    // facet-Jacobian terms: one value per node of every physical boundary
    // face, the six faces in one contiguous buffer, two parities
    const int nn[3] = {g.n0, g.n1, g.n2};
    int64_t tot = 0;
    for (int f = 0; f < 6; ++f) {
      const int ax = f >> 1, side = f & 1;
      g.fface[f] = nullptr;
      g.fn1[f] = g.fn2[f] = 0;
      g.ffoff[f] = -1;
      if (!g.bnd[ax][side]) continue;
      const int t1 = (ax == 0) ? 1 : 0, t2 = (ax == 2) ? 1 : 2;
      g.fn1[f] = nn[t1];
      g.fn2[f] = nn[t2];
      g.ffoff[f] = tot;
      tot += (int64_t)nn[t1] * nn[t2];
    }
    g.ffsize = tot;
    for (int q = 0; q < 2; ++q) {
      HIPC(hipMalloc(&ffbuf[q], sizeof(double) * (size_t)std::max<int64_t>(1, tot)));
      HIPC(hipMemsetAsync(ffbuf[q], 0, sizeof(double) * (size_t)std::max<int64_t>(1, tot), c->stream));
      g.ffbuf[q] = ffbuf[q];
    }
    for (int f = 0; f < 6; ++f) g.fface[f] = (g.ffoff[f] >= 0) ? ffbuf[0] + g.ffoff[f] : nullptr;
  }
  return TV_OK;
}

static int setup_mesh(Ctx* c, const tv_mesh_desc* m) {
  const int d = m->dim;
  if (d < 1 || d > 3) return c->fail(TV_ERR_ARG, "mesh dim must be 1..3");
  c->dim = d;
  c->coords.resize(d);
  for (int a = 0; a < d; ++a) {
    if (m->n_cells[a] < 1) return c->fail(TV_ERR_ARG, "n_cells must be >= 1 on every axis");
    if (!m->coords[a]) return c->fail(TV_ERR_ARG, "coords missing");
    c->coords[a].assign(m->coords[a], m->coords[a] + m->n_cells[a] + 1);
    for (int i = 0; i < m->n_cells[a]; ++i)
      if (!(c->coords[a][i + 1] > c->coords[a][i]))
        return c->fail(TV_ERR_ARG, "node coordinates must be strictly increasing");
  }
  if (!storage_perm(m, c->perm)) return c->fail(TV_ERR_ARG, "part_axis must be 1 (y) or 2 (z) for 3D meshes");
  c->n_parts = std::max(1, m->n_parts);
  c->part = m->part;
  if (c->part < 0 || c->part >= c->n_parts) return c->fail(TV_ERR_ARG, "part out of range");
  if (c->n_parts > 1 && (d == 1 || c->fam_T != TV_CG || c->fam_S != TV_CG))
    return c->fail(TV_ERR_ARG, "partitioned meshes require dim >= 2 and CG temperature and stress spaces");
  for (int s = 0; s < 3; ++s) {
    c->Ncell_glob[s] = (c->perm[s] < 0) ? 0 : m->n_cells[c->perm[s]];
    c->Nnode_glob[s] = c->Ncell_glob[s] + 1;
  }
  std::vector<double> tmp;
  if (c->fam_T == TV_CG) {
    const int N2 = c->Nnode_glob[2];
    const int P = c->n_parts, p = c->part;
    int b0, b1;
    part_planes(N2, P, p, &b0, &b1);
    if (b1 - b0 < 1) return c->fail(TV_ERR_ARG, "too many partitions for the mesh");
    c->plane_begin = b0;
    c->plane_end = b1;
    CgGrid& g = c->cg;
    std::vector<double> X[3];
    for (int s = 0; s < 3; ++s) X[s] = storage_coords(c, s, tmp);
    const int g_lo = (p > 0) ? 1 : 0, g_hi = (p < P - 1) ? 1 : 0;
    if (int e = build_cg_grid(c, d, X, b0 - g_lo, (b1 - b0) + g_lo + g_hi, g_lo, g_hi, p == 0, p == P - 1, g, c->coef,
                              &c->bnodes, c->ffbuf))
      return e;
    const int64_t plane = (int64_t)g.n0 * g.n1;
    c->nT = plane * g.n2;
    // the CG kernels index local nodes with 32-bit integers (68 M nodes = 290 GB
    // of state at materialize=1 would already exceed one MI355X)
    if (c->nT >= (int64_t)INT32_MAX) return c->fail(TV_ERR_ARG, "partition too large: >= 2^31 local nodes");
    c->ownT_off = plane * g.k_begin;
    c->ownT_n = plane * (g.k_end - g.k_begin);
    c->globT_off = plane * b0;
  } else {
    DgGrid& g = c->dg;
    g.c0 = c->Ncell_glob[0];
    g.c1 = std::max(1, c->Ncell_glob[1]);
    g.c2 = std::max(1, c->Ncell_glob[2]);
    g.k_begin = 0;
    g.k_end = g.c2;
    g.deg1 = (c->perm[1] < 0);
    g.deg2 = (c->perm[2] < 0);
    g.bnd[0][0] = g.bnd[0][1] = 1;
    g.bnd[1][0] = g.bnd[1][1] = g.deg1 ? 0 : 1;
    g.bnd[2][0] = g.bnd[2][1] = g.deg2 ? 0 : 1;
    const char* et = experiment_env("TVFEM_DG_TILE");
    const char* ec = experiment_env("TVFEM_DG_CHUNK");
    g.tile = et ? std::min(2, std::max(0, atoi(et))) : 2;  // 2: k_dg_tile with halo-loading edge waves
    g.tile_chunk = ec ? std::max(1, atoi(ec)) : 5;
    for (int s = 0; s < 3; ++s) {
      const std::vector<double>& X = storage_coords(c, s, tmp);
      std::vector<double> h;
      if (X.size() == 1) h.assign(1, 1.0);
      else for (size_t i = 0; i + 1 < X.size(); ++i) h.push_back(X[i + 1] - X[i]);
      const size_t nh = h.size();
      for (size_t q = 0; q < nh; ++q) h.push_back(1.0 / h[q]);  // [h..., 1/h...]
      HIPC(hipMalloc(&c->dgh[s], h.size() * sizeof(double)));
      HIPC(hipMemcpy(c->dgh[s], h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice));
      g.h[s] = c->dgh[s];
      g.ih[s] = c->dgh[s] + nh;
    }
    const int nl = 1 << d;
    c->nT = (int64_t)g.c0 * g.c1 * g.c2 * nl;
    c->ownT_off = 0;
    c->ownT_n = c->nT;
    c->globT_off = 0;
    c->plane_begin = 0;
    c->plane_end = g.c2;
  }
  // sigma space
  if (c->fam_S == c->fam_T) {
    c->nS = c->nT;
    c->ownS_off = c->ownT_off;
    c->ownS_n = c->ownT_n;
    c->globS_off = c->globT_off;
  } else {
    const int nl = 1 << d;
    const int64_t ncell = (int64_t)std::max(1, c->Ncell_glob[0]) * std::max(1, c->Ncell_glob[1]) *
                          std::max(1, c->Ncell_glob[2]);
    const int64_t nnode = (int64_t)c->Nnode_glob[0] * c->Nnode_glob[1] * c->Nnode_glob[2];
    c->nS = (c->fam_S == TV_CG) ? nnode : ncell * nl;
    c->ownS_off = 0;
    c->ownS_n = c->nS;
    c->globS_off = 0;
    // fem::interpolate: cells in order, last cell written wins at shared sigma dofs
    std::vector<int> map((size_t)c->nS, -1);
    const int C0 = std::max(1, c->Ncell_glob[0]), C1 = std::max(1, c->Ncell_glob[1]);
    const int N0 = c->Nnode_glob[0], N1 = c->Nnode_glob[1];
    const int act[3] = {0, c->perm[1] >= 0, c->perm[2] >= 0};
    for (int64_t cell = 0; cell < ncell; ++cell) {
      const int ci[3] = {(int)(cell % C0), (int)((cell / C0) % C1), (int)(cell / ((int64_t)C0 * C1))};
      for (int l = 0; l < nl; ++l) {
        int bits[3] = {0, 0, 0};
        int k = 0;
        for (int s = 0; s < 3; ++s) {
          if (s > 0 && !act[s]) continue;
          bits[s] = (l >> k) & 1;
          ++k;
        }
        const int64_t node = (int64_t)(ci[0] + bits[0]) + (int64_t)N0 * ((ci[1] + bits[1]) + (int64_t)N1 * (ci[2] + bits[2]));
        // DG dof numbering (cell-major) in device layout [l][cell]
        const int64_t dgdof = (int64_t)l * ncell + cell;
        if (c->fam_S == TV_CG) map[(size_t)node] = (int)dgdof;  // sigma CG <- T DG
        else map[(size_t)dgdof] = (int)node;                    // sigma DG <- T CG
      }
    }
    HIPC(hipMalloc(&c->map, sizeof(int) * (size_t)c->nS));
    HIPC(hipMemcpy(c->map, map.data(), sizeof(int) * (size_t)c->nS, hipMemcpyHostToDevice));
  }
  // thermal constants
  const tv_params& P = c->P;
  for (CgGrid* g = &c->cg; g; g = nullptr) {
    g->dt = P.dt; g->dt_alpha = P.dt * P.alpha; g->dt_f = P.dt * P.f;
    g->a_rad = 0.001 * (P.sigma * P.epsilon); g->a_conv = 0.001 * P.htc;
    g->T_amb = P.T_ambient; g->T_amb4 = P.T_ambient * P.T_ambient * P.T_ambient * P.T_ambient;
  }
  {
    DgGrid* g = &c->dg;
    g->dt = P.dt; g->dt_alpha = P.dt * P.alpha; g->dt_f = P.dt * P.f;
    g->a_rad = 0.001 * (P.sigma * P.epsilon); g->a_conv = 0.001 * P.htc;
    g->T_amb = P.T_ambient; g->T_amb4 = P.T_ambient * P.T_ambient * P.T_ambient * P.T_ambient;
    g->penalty = 5.0;
  }
  return TV_OK;
}

constexpr int64_t kCgsAutoMaxNodes = 3000000;  // AUTO Krylov form: single reduction up to this slab size

static int setup_fields(Ctx* c) {
  const int d = c->dim, dd = d * d;
  const bool all = c->O.materialize != 0;
  int rc;
#define AF(id, sp, bs) if ((rc = alloc_field(c, id, sp, bs)) != TV_OK) return rc
  AF(TV_F_T, 0, 1);
  AF(TV_F_T_PREV, 0, 1);
  AF(TV_F_TF, 0, 1);
  AF(TV_F_TF_PARTIAL, 0, 6);
  AF(TV_F_PHI, 0, 1);
  AF(TV_F_XI, 0, 1);
  AF(TV_F_S_TILDE, 1, 6 * dd);
  AF(TV_F_SIGMA_TILDE, 1, 6 * dd);
  AF(TV_F_SIGMA, 1, dd);
  const bool paper = c->O.model_mode == TV_MODEL_PAPER;
  if (paper && !all) {  // s / sigma partial feed s~ / sigma~ (Eq. 16): state in paper mode
    AF(TV_F_S_PARTIAL, 1, 6 * dd);
    AF(TV_F_SIGMA_PARTIAL, 1, 6 * dd);
    alias_field(c, TV_F_S_PARTIAL_NEXT, TV_F_S_PARTIAL);
    alias_field(c, TV_F_SIGMA_PARTIAL_NEXT, TV_F_SIGMA_PARTIAL);
  }
  if (paper && c->fam_T != c->fam_S) HIPC(hipMalloc(&c->Tfo, sizeof(double) * (size_t)std::max<int64_t>(1, c->nT)));
  if (all) {
    AF(TV_F_T_NEXT, 0, 1);
    AF(TV_F_PHI_NEXT, 0, 1);
    AF(TV_F_THERMAL_STRAIN, 1, dd);
    AF(TV_F_TOTAL_STRAIN, 1, dd);
    AF(TV_F_DEVIATORIC_STRAIN, 1, dd);
    AF(TV_F_DS_PARTIAL, 1, 6 * dd);
    AF(TV_F_DSIGMA_PARTIAL, 1, 6 * dd);
    AF(TV_F_S_PARTIAL, 1, 6 * dd);
    AF(TV_F_SIGMA_PARTIAL, 1, 6 * dd);
    alias_field(c, TV_F_S_PARTIAL_NEXT, TV_F_S_PARTIAL);
    alias_field(c, TV_F_SIGMA_PARTIAL_NEXT, TV_F_SIGMA_PARTIAL);
  }
#undef AF
  alias_field(c, TV_F_TF_PREV, TV_F_TF);
  alias_field(c, TV_F_TF_PARTIAL_PREV, TV_F_TF_PARTIAL);
  alias_field(c, TV_F_S_TILDE_NEXT, TV_F_S_TILDE);
  alias_field(c, TV_F_SIGMA_TILDE_NEXT, TV_F_SIGMA_TILDE);
  // PCG work vectors (T space, local size)
  const size_t nb = sizeof(double) * (size_t)std::max<int64_t>(1, c->nT);
  HIPC(hipMalloc(&c->r, nb));
  HIPC(hipMalloc(&c->z, nb));
  HIPC(hipMalloc(&c->pA, nb));
  HIPC(hipMalloc(&c->pB, nb));
  HIPC(hipMalloc(&c->w, nb));
  HIPC(hipMalloc(&c->dinv, nb));
  for (double* p : {c->r, c->z, c->pA, c->pB, c->w, c->dinv}) HIPC(hipMemsetAsync(p, 0, nb, c->stream));
  c->f[TV_F_RESIDUAL].ptr = c->r; c->f[TV_F_RESIDUAL].bs = 1; c->f[TV_F_RESIDUAL].space = 0;
  if (int e = alloc_field(c, TV_F_DX, 0, 1)) return e;
  int np = kVecBlocksMax;
  if (c->um) np = std::max(np, um_num_blocks(c->umg));
  else if (c->fam_T == TV_CG) np = std::max(np, cg_num_blocks(c->cg, true));
  else np = std::max(np, dg_num_blocks(c->dg));
  c->n_partials_cap = np;
  // records of width <= 3 per workgroup + the shard records of the two-level tail
  HIPC(hipMalloc(&c->partials, sizeof(double) * 3 * ((size_t)np + 2 * kShards)));
  HIPC(hipMalloc(&c->sums, sizeof(double) * 8));
  HIPC(hipMalloc(&c->counters, sizeof(unsigned) * kCounterWords));
  HIPC(hipMemsetAsync(c->counters, 0, sizeof(unsigned) * kCounterWords, c->stream));
  HIPC(hipMalloc(&c->st, sizeof(PcgState)));
  HIPC(hipMalloc(&c->tflag, sizeof(int)));
  HIPC(hipMemsetAsync(c->tflag, 0, sizeof(int), c->stream));  // the tilde fields start at +0.0
  HIPC(hipHostMalloc(&c->h_st, 3 * sizeof(PcgState)));
  for (int k = 0; k < 2; ++k) HIPC(hipEventCreateWithFlags(&c->evp[k], hipEventDisableTiming));
  HIPC(hipHostMalloc(&c->h_sums, sizeof(double) * 8));
  const int var = c->O.pcg_variant;
  const bool can = c->fam_T == TV_CG && !c->um && cg_cgs_supported(c->cg);
  if (var == TV_PCG_SINGLE_REDUCTION && !can)
    return c->fail(TV_ERR_ARG, "pcg_variant SINGLE_REDUCTION needs a 3D CG1 temperature space");
  // AUTO: the single-reduction form where the mesh is partitioned into slabs
  // of at most kCgsAutoMaxNodes owned nodes (one RCCL group per iteration
  // instead of two all-reduces + a halo + two logic launches); on one
  // partition, and on larger slabs where its heavier launch is bandwidth-bound,
  // KSPCG's two lighter launches are faster (measured on the C4 per-rank
  // shares, DESIGN.md §5: 4.1M nodes 13.2 vs 18.3 ms/step, against ~2.7 ms of
  // communication the single reduction saves; 2M nodes 7.6 vs 8.6 ms; 1M
  // nodes 6.5 vs 6.7 ms)
  c->cgs = can && (var == TV_PCG_SINGLE_REDUCTION ||
                   (var == TV_PCG_AUTO && c->n_parts > 1 && c->ownT_n <= kCgsAutoMaxNodes));
  if (c->cgs) {
    for (double** q : {&c->cr[0], &c->cr[1], &c->cs[0], &c->cs[1], &c->cw1}) {
      HIPC(hipMalloc(q, nb));
      HIPC(hipMemsetAsync(*q, 0, nb, c->stream));
    }
    const size_t plane = (size_t)c->cg.n0 * c->cg.n1;
    HIPC(hipMalloc(&c->wsend, sizeof(double) * 2 * plane));
  }
  return TV_OK;
}

// --------------------------------------------------------------------------------------
// field transfer: reference interleaved layout <-> device component-major layout
// --------------------------------------------------------------------------------------
__global__ void k_interleave(int dir, double* __restrict__ buf, double* __restrict__ dev, int64_t ndof, int bs,
                             int64_t stride, int64_t off, int dg_nl, int64_t dg_ncell) {
  // dir 0: buf (host layout, dof*bs+comp) -> dev ; dir 1: dev -> buf
  const int64_t total = ndof * bs;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t dof = t / bs;
    const int comp = (int)(t % bs);
    int64_t di = (dg_nl > 0) ? (dof % dg_nl) * dg_ncell + dof / dg_nl : off + dof;
    double* p = dev + comp * stride + di;
    if (dir == 0) *p = buf[t];
    else buf[t] = *p;
  }
}

static int transfer(Ctx* c, int field, double* host, size_t n, int dir) {
  if (field < 0 || field >= TV_NUM_FIELDS) return c->fail(TV_ERR_ARG, "bad field id");
  FieldInfo& fi = c->f[field];
  if (!fi.ptr) return c->fail(TV_ERR_STATE, "field not materialized (options.materialize = 0 keeps state fields only)");
  const int64_t ndof = (fi.space == 0) ? c->ownT_n : c->ownS_n;
  const int64_t off = (fi.space == 0) ? c->ownT_off : c->ownS_off;
  const int64_t stride = (fi.space == 0) ? c->nT : c->nS;
  const size_t need = (size_t)ndof * fi.bs;
  if (n != need)
    return c->fail(TV_ERR_ARG, "size mismatch: expected " + std::to_string(need) + " values, got " + std::to_string(n));
  const bool dgsp = (fi.space == 0 ? c->fam_T : c->fam_S) == TV_DG;
  const int nl = dgsp ? (1 << c->dim) : 0;
  const int64_t ncell = dgsp ? ndof / nl : 0;
  const size_t bytes = need * sizeof(double);
  if (c->scratch_bytes < bytes) {
    if (c->scratch) HIPC(hipFree(c->scratch));
    c->scratch = nullptr;
    HIPC(hipMalloc(&c->scratch, std::max<size_t>(bytes, 8)));
    c->scratch_bytes = bytes;
  }
  const int blocks = (int)std::min<int64_t>(std::max<int64_t>(1, ((int64_t)need + 255) / 256), 16384);
  if (dir == 0) {
    const bool tilde = field == TV_F_S_TILDE || field == TV_F_S_TILDE_NEXT || field == TV_F_SIGMA_TILDE ||
                       field == TV_F_SIGMA_TILDE_NEXT;
    if (tilde) {  // values other than +0.0 end the all-zero tracking of the tilde fields
      const uint64_t* b = reinterpret_cast<const uint64_t*>(host);
      uint64_t any = 0;
      for (size_t k = 0; k < need; ++k) any |= b[k];
      if (any) {
        static const int one = 1;
        HIPC(hipMemcpyAsync(c->tflag, &one, sizeof(int), hipMemcpyHostToDevice, c->stream));
      }
    }
    HIPC(hipMemcpyAsync(c->scratch, host, bytes, hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(k_interleave, dim3(blocks), dim3(256), 0, c->stream, 0, c->scratch, fi.ptr, ndof, fi.bs,
                       stride, off, nl, ncell);
    HIPC(hipGetLastError());
    HIPC(hipStreamSynchronize(c->stream));
  } else {
    hipLaunchKernelGGL(k_interleave, dim3(blocks), dim3(256), 0, c->stream, 1, c->scratch, fi.ptr, ndof, fi.bs,
                       stride, off, nl, ncell);
    HIPC(hipGetLastError());
    HIPC(hipMemcpyAsync(host, c->scratch, bytes, hipMemcpyDeviceToHost, c->stream));
    HIPC(hipStreamSynchronize(c->stream));
  }
  return TV_OK;
}

// --------------------------------------------------------------------------------------
// communication
// --------------------------------------------------------------------------------------
static bool multi_rank(const Ctx* c) { return c->nranks > 1 && (c->comm || c->host_sendrecv); }

static int halo_host(Ctx* c, double* v) {
  const CgGrid& g = c->cg;
  const int64_t plane = (int64_t)g.n0 * g.n1;
  double* s_lo = c->h_halo;
  double* s_hi = c->h_halo + plane;
  double* r_lo = c->h_halo + 2 * plane;
  double* r_hi = c->h_halo + 3 * plane;
  if (g.g_lo) HIPC(hipMemcpyAsync(s_lo, v + plane * g.k_begin, plane * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  if (g.g_hi) HIPC(hipMemcpyAsync(s_hi, v + plane * (g.k_end - 1), plane * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPC(hipStreamSynchronize(c->stream));
  if (g.g_lo && c->host_sendrecv(s_lo, (size_t)plane, c->rank - 1, r_lo, (size_t)plane, c->rank - 1, c->host_user))
    return c->fail(TV_ERR_COMM, "host sendrecv failed");
  if (g.g_hi && c->host_sendrecv(s_hi, (size_t)plane, c->rank + 1, r_hi, (size_t)plane, c->rank + 1, c->host_user))
    return c->fail(TV_ERR_COMM, "host sendrecv failed");
  if (g.g_lo) HIPC(hipMemcpyAsync(v, r_lo, plane * sizeof(double), hipMemcpyHostToDevice, c->stream));
  if (g.g_hi) HIPC(hipMemcpyAsync(v + plane * g.k_end, r_hi, plane * sizeof(double), hipMemcpyHostToDevice, c->stream));
  HIPC(hipStreamSynchronize(c->stream));
  return TV_OK;
}

static int halo(Ctx* c, double* v) {
  if (!multi_rank(c) || c->fam_T != TV_CG) return TV_OK;
  if (c->host_sendrecv) return halo_host(c, v);
  const CgGrid& g = c->cg;
  const int64_t plane = (int64_t)g.n0 * g.n1;
  NCCLC(ncclGroupStart());
  if (g.g_lo) {  // neighbour rank-1: send first owned plane, receive ghost plane 0
    NCCLC(ncclSend(v + plane * g.k_begin, plane, ncclDouble, c->rank - 1, c->comm, c->stream));
    NCCLC(ncclRecv(v, plane, ncclDouble, c->rank - 1, c->comm, c->stream));
  }
  if (g.g_hi) {
    NCCLC(ncclSend(v + plane * (g.k_end - 1), plane, ncclDouble, c->rank + 1, c->comm, c->stream));
    NCCLC(ncclRecv(v + plane * g.k_end, plane, ncclDouble, c->rank + 1, c->comm, c->stream));
  }
  NCCLC(ncclGroupEnd());
  return TV_OK;
}

static int allreduce(Ctx* c, double* v, int n) {
  if (!multi_rank(c)) return TV_OK;
  if (c->host_allreduce) {
    HIPC(hipMemcpyAsync(c->h_sums + 4, v, n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPC(hipStreamSynchronize(c->stream));
    if (c->host_allreduce(c->h_sums + 4, n, c->host_user)) return c->fail(TV_ERR_COMM, "host allreduce failed");
    HIPC(hipMemcpyAsync(v, c->h_sums + 4, n * sizeof(double), hipMemcpyHostToDevice, c->stream));
    return TV_OK;
  }
  NCCLC(ncclAllReduce(v, v, n, ncclDouble, ncclSum, c->comm, c->stream));
  return TV_OK;
}

// reduce partial records -> (allreduce) -> scalar logic
static int reduce_logic(Ctx* c, int n, int W, int kind, int check_done) {
  if (!multi_rank(c)) {
    launch_reduce_logic(c->partials, n, W, c->sums, c->st, kind, check_done, c->stream);
  } else {
    launch_reduce_logic(c->partials, n, W, c->sums, c->st, 0, 0, c->stream);
    if (int e = allreduce(c, c->sums, W)) return e;
    if (kind) launch_logic(c->st, c->sums, kind, c->stream);
  }
  return TV_OK;
}

// --------------------------------------------------------------------------------------
// operators
// --------------------------------------------------------------------------------------
static void op_residual(Ctx* c, const double* T, const double* Tp, double* F) {
  if (c->um) launch_um_residual(c->umg, T, Tp, F, c->stream);
  else if (c->fam_T == TV_CG) launch_cg_residual(c->cg, T, Tp, F, c->stream);
  else launch_dg_residual(c->dg, T, Tp, F, c->stream);
}
static void op_diag(Ctx* c, const double* T, double* d, int invert) {
  // Jacobian "assembly": the diagonal for the Jacobi PC (J(T) itself is matrix-free)
  if (c->um) launch_um_diag(c->umg, T, d, invert, c->stream);
  else if (c->fam_T == TV_CG) launch_cg_diag(c->cg, T, d, invert, c->stream);
  else launch_dg_diag(c->dg, T, d, invert, c->stream);
}
static void op_japply(Ctx* c, const double* T, const double* x, double* y, double* partials, int* np) {
  if (c->um) launch_um_japply(c->umg, T, x, y, c->stream);
  else if (c->fam_T == TV_CG) launch_cg_japply(c->cg, T, x, y, partials, np, c->stream);
  else launch_dg_japply(c->dg, T, x, y, partials, np, c->stream);
}
static bool op_japply_fused(Ctx* c, const double* T, int* np, const RedTail* tail = nullptr, int it = 0) {
  if (c->um) {  // p <- z + b p, w <- J p, p.w and the reduction tail in one launch
    *np = launch_um_japply_fused(c->umg, T, c->z, c->pA, c->pB, c->w, c->st, c->partials, it, tail, c->stream);
    return tail && tail->counter;
  }
  if (c->fam_T == TV_CG)
    return launch_cg_japply_fused(c->cg, T, c->z, c->pA, c->pB, c->w, c->st, c->partials, np, c->stream, tail, it);
  return launch_dg_japply_fused(c->dg, T, c->z, c->pA, c->pB, c->w, c->st, c->partials, np, c->stream, tail);
}

// --------------------------------------------------------------------------------------
// Jacobi-PCG for J(T) dx = r  (PETSc KSPCG restated; see tv_pcg.hip)
// --------------------------------------------------------------------------------------
// it: index of this iteration within the solve (the device counter st->it
// equals it until convergence, after which every kernel exits at once)
constexpr int kTsCap = 1 << 15;

// reads the pending timestamp slots back and adds them to the stats
static int ts_flush(Ctx* c) {
  if (!c->d_ts) return TV_OK;
  if (!c->ts_pending.empty()) {
    std::vector<uint64_t> h((size_t)4 * c->ts_next);
    HIPC(hipMemcpyAsync(h.data(), c->d_ts, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    HIPC(hipStreamSynchronize(c->stream));
    for (int sl : c->ts_pending) {
      const uint64_t* t = &h[(size_t)4 * sl];
      for (int k = 0; k < 2; ++k) {
        if (t[2 * k] == 0 || t[2 * k + 1] < t[2 * k]) continue;  // launch without a timed tail
        c->ksum[k] += (double)(t[2 * k + 1] - t[2 * k]) / c->ts_khz;
        c->kcnt[k] += 1;
      }
    }
    c->ts_pending.clear();
  }
  c->ts_next = 0;
  HIPC(hipMemsetAsync(c->d_ts, 0, (size_t)4 * kTsCap * sizeof(uint64_t), c->stream));
  return TV_OK;
}

static int pcg_iteration(Ctx* c, const double* T, int it) {
  const int64_t off = c->ownT_off, n = c->ownT_n;
  // timestamp slot of this iteration (see ts_flush); the matvec launchers
  // without a reduction tail (DG, 1D/2D CG) leave theirs at 0
  const int slot = c->ts_next + it;
  uint64_t* ts = (c->ktime && (it % c->kstride) == 0 && slot < kTsCap) ? c->d_ts + 4 * slot : nullptr;
  const bool multi = multi_rank(c);
  // single GPU: the last-arriving workgroup of each launch reduces the partial
  // records and runs the KSPCG scalar logic in-kernel (no separate reduce
  // launch); multi-GPU: it only reduces, RCCL all-reduces, then the logic runs.
  RedTail t1{c->counters, c->partials, c->sums, c->st, multi ? 0 : 2, ts};
  int np = 0;
  const bool fused1 = op_japply_fused(c, T, &np, &t1, it);  // p <- z + b p ; w <- J p ; p.w
  if (!fused1) {
    if (int e = reduce_logic(c, np, 1, 2, 1)) return e;  // dpi, a
  } else if (multi) {
    if (int e = allreduce(c, c->sums, 1)) return e;
    launch_logic(c->st, c->sums, 2, c->stream);
  }
  RedTail t2{c->counters + kTailCounters, c->partials, c->sums, c->st, multi ? 0 : 3, ts ? ts + 2 : nullptr};
  const FaceAdd fa = (c->fam_T == TV_CG && !c->um) ? cg_face_add(c->cg, off) : FaceAdd{};
  launch_pcg_update(n, c->st, c->pA + off, c->pB + off, c->w + off, c->dinv + off, c->f[TV_F_DX].ptr + off,
                    c->z + off, c->partials, c->stream, &t2, &fa, it);
  if (multi) {  // dp, beta, convergence
    if (int e = allreduce(c, c->sums, 2)) return e;
    launch_logic(c->st, c->sums, 3, c->stream);
  }
  if (int e = halo(c, c->z)) return e;
  return TV_OK;
}

static int pcg_solve(Ctx* c, const double* T, int* its, int* reason) {
  const int64_t off = c->ownT_off, n = c->ownT_n;
  // state init
  PcgState h{};
  h.rtol = c->O.ksp_rtol;
  h.atol = c->O.ksp_atol;
  h.dtol = c->O.ksp_dtol;
  h.max_it = c->O.ksp_max_it;
  // from pinned memory (an asynchronous upload; a pageable source is staged by
  // the runtime -- no step-time change measured at C2 / C3 / C4)
  c->h_st[2] = h;
  HIPC(hipMemcpyAsync(c->st, &c->h_st[2], sizeof(PcgState), hipMemcpyHostToDevice, c->stream));
  launch_pcg_init(n, c->r + off, c->dinv + off, c->z + off, c->f[TV_F_DX].ptr + off, c->partials, c->stream);
  if (int e = reduce_logic(c, pcg_vec_blocks(n), 2, 1, 0)) return e;
  if (int e = halo(c, c->z)) return e;
  if (c->ktime && c->ts_next + c->O.ksp_max_it + 4 * c->O.pcg_batch + 8 > kTsCap)
    if (int e = ts_flush(c)) return e;
  // Batches of iterations are queued one ahead of the convergence poll: while
  // the host waits for the state copied at the end of batch k, batch k + 1 is
  // already in the stream, so the GPU never idles on the host's turnaround.
  // After convergence the queued launches exit at their first instruction.
  int launched = 0, slot = 0;
  auto enqueue = [&](int nb, int k) -> int {
    for (int b = 0; b < nb; ++b)
      if (int e = pcg_iteration(c, T, launched + b)) return e;
    launched += nb;
    HIPC(hipGetLastError());
    HIPC(hipMemcpyAsync(&c->h_st[k], c->st, sizeof(PcgState), hipMemcpyDeviceToHost, c->stream));
    HIPC(hipEventRecord(c->evp[k], c->stream));
    return TV_OK;
  };
  // batches queued behind the first: pcg_batch / 8 iterations (1 by default);
  // the host's turnaround (~30 us) is well inside one iteration (~130 us at C4),
  // and every iteration queued past convergence costs two early-exit launches
  static int div = -1;
  if (div < 0) {
    const char* e = experiment_env("TVFEM_PCG_SMALL_DIV");
    div = e ? std::max(1, atoi(e)) : 8;
  }
  const int small = std::max(1, c->O.pcg_batch / div);
  if (int e = enqueue(std::max(1, c->pcg_hint > 4 ? c->pcg_hint - 3 : c->O.pcg_batch), 0)) return e;
  for (;;) {
    if (int e = enqueue(small, slot ^ 1)) return e;
    HIPC(hipEventSynchronize(c->evp[slot]));
    if (c->h_st[slot].done) break;
    if (launched > c->O.ksp_max_it + 2 * small + 2) return c->fail(TV_ERR_KSP, "PCG: iteration guard exceeded");
    slot ^= 1;
  }
  // (the batch queued behind the converged one exits early; stream order covers it)
  *its = c->h_st[slot].it;
  *reason = c->h_st[slot].reason;
  launch_pcg_dx_tail(n, c->st, c->pA + off, c->pB + off, c->f[TV_F_DX].ptr + off, *its, c->stream);
  c->pcg_hint = c->h_st[slot].it;
  if (c->ktime) {  // productive iterations only (launches queued behind convergence exit at once)
    for (int it = 0; it < *its; it += c->kstride)
      if (c->ts_next + it < kTsCap) c->ts_pending.push_back(c->ts_next + it);
    c->ts_next = std::min(kTsCap, c->ts_next + launched);
  }
  return TV_OK;
}

// ---- geometric-multigrid preconditioned CG (options.preconditioner = GMG) ----
// Gershgorin bound of D^-1 J on a rectilinear level: max over nodes of the
// exact absolute row sum of the 27-point cell operator M + dt alpha K over its
// diagonal (the tensor-product entries from the per-axis 1D rows), over the
// distinct (row_x, row_y, row_z) combinations only.  The Robin facet rows are
// facet masses (row sum / diagonal <= 2.25 for Q1 facets): floor 2.25, then 5 %.
static double mg_gershgorin(const std::vector<double> (&X)[3], double dt_alpha) {
  using Row = std::array<double, 6>;  // M lo / di / up, K lo / di / up
  std::vector<Row> rows[3];
  for (int s = 0; s < 3; ++s) {
    std::vector<double> cf;
    axis_coefs(X[s], 0, (int)X[s].size(), cf);
    for (size_t i = 0; i < X[s].size(); ++i) {
      const double* c = &cf[i * C_NCOEF];
      rows[s].push_back({c[C_MLO], c[C_MDI], c[C_MUP], c[C_KLO], c[C_KDI], c[C_KUP]});
    }
    std::sort(rows[s].begin(), rows[s].end());
    rows[s].erase(std::unique(rows[s].begin(), rows[s].end()), rows[s].end());
  }
  double b = 0.0;
  for (const Row& r0 : rows[0])
    for (const Row& r1 : rows[1])
      for (const Row& r2 : rows[2]) {
        double sum = 0.0, diag = 0.0;
        for (int a = 0; a < 3; ++a)
          for (int bb = 0; bb < 3; ++bb)
            for (int cc = 0; cc < 3; ++cc) {
              const double v = r0[a] * r1[bb] * r2[cc] +
                               dt_alpha * (r0[3 + a] * r1[bb] * r2[cc] + r0[a] * r1[3 + bb] * r2[cc] +
                                           r0[a] * r1[bb] * r2[3 + cc]);
              sum += std::fabs(v);
              if (a == 1 && bb == 1 && cc == 1) diag = v;
            }
        b = std::max(b, sum / diag);
      }
  return std::max(b, 2.25) * 1.05;
}

template <class T>
static int mg_upload(Ctx* c, MgLevel& L, const std::vector<T>& h, const T** out) {
  void* p = nullptr;
  HIPC(hipMalloc(&p, sizeof(T) * std::max<size_t>(1, h.size())));
  L.bufs.push_back(p);
  HIPC(hipMemcpy(p, h.data(), sizeof(T) * h.size(), hipMemcpyHostToDevice));
  *out = static_cast<const T*>(p);
  return TV_OK;
}

static double mg_omega(double b) { return 2.0 / (1.1 * b); }

// Coarse levels up to this many nodes run the x-row stencil kernel (facet terms
// inline: one launch per J x instead of march + k_cg_addfaces, no FaceAdd in
// the consumers); TVFEM_MG_ROWK=<nodes> overrides it (experiments, 0 = march)
static int64_t mg_rows_kernel_nodes() {
  static const int64_t v = [] {
    const char* e = experiment_env("TVFEM_MG_ROWK");
    return e ? (int64_t)atoll(e) : (int64_t)0;
  }();
  return v;
}

// the hierarchy below the fine grid (single partition, 3D CG1 marching path)
// the CG1 level of the box given by X (single partition), its vectors and weight
static int mg_add_cg_level(Ctx* c, const std::vector<double> (&X)[3], double da) {
  c->mg.emplace_back();
  MgLevel& L = c->mg.back();
  for (int s = 0; s < 3; ++s) L.X[s] = X[s];
  if (int e = build_cg_grid(c, 3, L.X, 0, (int)L.X[2].size(), 0, 0, true, true, L.g, L.coef, &L.bnodes, L.ffbuf))
    return e;
  const CgGrid& f = c->cg;  // thermal constants (set by setup_fields for both families)
  L.g.dt = f.dt; L.g.dt_alpha = f.dt_alpha; L.g.dt_f = f.dt_f;
  L.g.a_rad = f.a_rad; L.g.a_conv = f.a_conv; L.g.T_amb = f.T_amb; L.g.T_amb4 = f.T_amb4;
  L.n = (int64_t)L.g.n0 * L.g.n1 * L.g.n2;
  L.g.rows_kernel = L.n <= mg_rows_kernel_nodes() ? 1 : 0;
  for (double** q : {&L.T, &L.b, &L.x, &L.w, &L.dinv}) {
    void* p = nullptr;
    HIPC(hipMalloc(&p, sizeof(double) * (size_t)L.n));
    HIPC(hipMemsetAsync(p, 0, sizeof(double) * (size_t)L.n, c->stream));
    L.bufs.push_back(p);
    *q = static_cast<double*>(p);
  }
  L.omega = mg_omega(mg_gershgorin(L.X, da));
  return TV_OK;
}

// lambda_max(B^-1 J) of the DG1 operator by power iteration, B the cell blocks
// (point Jacobi D under the experiment switch); SIPG rows have no closed-form
// Gershgorin bound here.  The smoother takes it with a 21 % margin
static int mg_dg_lambda(Ctx* c, double* lam) {
  const int64_t n = c->nT;
  const double* T = c->f[TV_F_T].ptr;
  std::vector<double> h((size_t)n);
  uint64_t st = 0x9E3779B97F4A7C15ull;
  double nrm = 0.0;
  for (int64_t t = 0; t < n; ++t) {  // fixed-seed xorshift start vector in (0.5, 1.5)
    st ^= st << 13; st ^= st >> 7; st ^= st << 17;
    h[(size_t)t] = 0.5 + (double)(st >> 11) * (1.0 / 9007199254740992.0);
    nrm += h[(size_t)t] * h[(size_t)t];
  }
  for (double& v : h) v /= std::sqrt(nrm);
  HIPC(hipMemcpyAsync(c->mgx, h.data(), sizeof(double) * (size_t)n, hipMemcpyHostToDevice, c->stream));
  if (c->dggface) launch_dg_gface(c->dg, T, c->dggface, c->stream);
  else launch_dg_diag(c->dg, T, c->dinv, 1, c->stream);
  std::vector<double> part(1024);
  double l = 0.0;
  for (int it = 0; it < 30; ++it) {
    op_japply(c, T, c->mgx, c->w, nullptr, nullptr);
    if (c->dggface) launch_dg_bsmooth(c->dg, nullptr, c->w, nullptr, c->dggface, 1.0, c->w, 0, c->stream);  // in place, per cell
    const int nb = launch_mg_pow(n, c->dggface ? nullptr : c->dinv, c->w, c->partials, c->stream);
    HIPC(hipMemcpyAsync(part.data(), c->partials, sizeof(double) * (size_t)nb, hipMemcpyDeviceToHost, c->stream));
    HIPC(hipStreamSynchronize(c->stream));
    double s2 = 0.0;
    for (int b = 0; b < nb; ++b) s2 += part[(size_t)b];
    l = std::sqrt(s2);  // ||D^-1 J x|| with ||x|| = 1
    if (!(l > 0.0) || !std::isfinite(l)) return c->fail(TV_ERR_HIP, "GMG: DG eigenvalue estimate failed");
    launch_mg_scale(n, c->w, 1.0 / l, c->mgx, c->stream);
  }
  *lam = l;
  return TV_OK;
}

static int mg_setup(Ctx* c) {
  const bool dg = c->fam_T == TV_DG;
  if (c->dim != 3 || c->um || (!dg && !cg_cgs_supported(c->cg)) || (dg && (c->dg.deg1 || c->dg.deg2)))
    return c->fail(TV_ERR_ARG, "preconditioner GMG: 3D CG1 or DG1 temperature space on a rectilinear mesh only");
  if (c->n_parts > 1) return c->fail(TV_ERR_ARG, "preconditioner GMG: one partition (use TV_PC_JACOBI when partitioned)");
  if (c->cgs) return c->fail(TV_ERR_ARG, "preconditioner GMG runs in the KSPCG form (pcg_variant KSPCG or AUTO)");
  std::vector<double> tmp, Xf[3];
  for (int s = 0; s < 3; ++s) Xf[s] = storage_coords(c, s, tmp);
  const double da = c->P.dt * c->P.alpha;
  HIPC(hipMalloc(&c->mgx, sizeof(double) * (size_t)std::max<int64_t>(1, c->nT)));
  HIPC(hipMemsetAsync(c->mgx, 0, sizeof(double) * (size_t)std::max<int64_t>(1, c->nT), c->stream));
  if (dg) {
    // level 1: the CG1 space of the same box (two-level DG -> CG, then the CG hierarchy)
    c->mg_dg = true;
    if (!experiment_env("TVFEM_MG_DG_POINT")) {
      HIPC(hipMalloc(&c->dggface, sizeof(double) * (size_t)dg_gface_size(c->dg)));
    }
    double lam = 0.0;
    if (int e = mg_dg_lambda(c, &lam)) return e;
    c->mg_omega0 = 2.0 / (1.1 * 1.1 * lam);
    if (int e = mg_add_cg_level(c, Xf, da)) return e;
  } else {
    c->mg_omega0 = mg_omega(mg_gershgorin(Xf, da));
  }
  const int max_levels = c->O.mg_levels > 0 ? c->O.mg_levels : 8;
  const bool automatic = c->O.mg_levels <= 0;
  std::vector<double> Xp[3] = {Xf[0], Xf[1], Xf[2]};
  for (int lev = 1 + (dg ? 1 : 0); lev < max_levels; ++lev) {
    double h = 1e300;  // smallest mean cell length over the axes
    bool coarsen[3], any = false;
    for (int s = 0; s < 3; ++s) {
      const int cells = (int)Xp[s].size() - 1;
      coarsen[s] = cells >= 2;
      any = any || coarsen[s];
      if (cells >= 1) h = std::min(h, (Xp[s].back() - Xp[s].front()) / cells);
    }
    // stop where the operator is mass-dominated: a Jacobi step is then a good solve
    if (!any || (automatic && da / (h * h) <= 0.5)) break;
    c->mg.emplace_back();
    MgLevel& L = c->mg.back();
    std::vector<char> is_c[3];  // fine node kept on this level
    for (int s = 0; s < 3; ++s) {
      const int nf = (int)Xp[s].size();
      is_c[s].assign(nf, 1);
      if (!coarsen[s]) {
        L.X[s] = Xp[s];
        continue;
      }
      // every other node, and the last one (an odd cell count keeps one fine cell at the end)
      for (int i = 0; i < nf; ++i) is_c[s][i] = (i % 2 == 0 || i == nf - 1) ? 1 : 0;
      for (int i = 0; i < nf; ++i)
        if (is_c[s][i]) L.X[s].push_back(Xp[s][i]);
    }
    if (int e = build_cg_grid(c, 3, L.X, 0, (int)L.X[2].size(), 0, 0, true, true, L.g, L.coef, &L.bnodes, L.ffbuf))
      return e;
    const CgGrid& f = c->cg;
    L.g.dt = f.dt; L.g.dt_alpha = f.dt_alpha; L.g.dt_f = f.dt_f;
    L.g.a_rad = f.a_rad; L.g.a_conv = f.a_conv; L.g.T_amb = f.T_amb; L.g.T_amb4 = f.T_amb4;
    L.n = (int64_t)L.g.n0 * L.g.n1 * L.g.n2;
    L.g.rows_kernel = L.n <= mg_rows_kernel_nodes() ? 1 : 0;
    for (double** q : {&L.T, &L.b, &L.x, &L.w, &L.dinv}) {
      void* p = nullptr;
      HIPC(hipMalloc(&p, sizeof(double) * (size_t)L.n));
      HIPC(hipMemsetAsync(p, 0, sizeof(double) * (size_t)L.n, c->stream));
      L.bufs.push_back(p);
      *q = static_cast<double*>(p);
    }
    L.omega = mg_omega(mg_gershgorin(L.X, da));
    // transfer maps (finer level Xp -> this level)
    MgXfer& x = L.xf;
    for (int s = 0; s < 3; ++s) {
      const int nf = (int)Xp[s].size(), nc = (int)L.X[s].size();
      std::vector<int> pi(2 * (size_t)nf), ri(3 * (size_t)nc), cpos(nf, -1), fpos;
      std::vector<double> pw(2 * (size_t)nf, 0.0), rw(3 * (size_t)nc, 0.0);
      for (int i = 0; i < nf; ++i)
        if (is_c[s][i]) {
          cpos[i] = (int)fpos.size();
          fpos.push_back(i);
        }
      for (int i = 0; i < nf; ++i) {
        if (is_c[s][i]) {
          pi[2 * i] = pi[2 * i + 1] = cpos[i];
          pw[2 * i] = 1.0;
        } else {  // linear interpolation between the coarse neighbours i - 1 and i + 1
          const double wl = (Xp[s][i + 1] - Xp[s][i]) / (Xp[s][i + 1] - Xp[s][i - 1]);
          pi[2 * i] = cpos[i - 1];
          pi[2 * i + 1] = cpos[i + 1];
          pw[2 * i] = wl;
          pw[2 * i + 1] = 1.0 - wl;
        }
      }
      for (int I = 0; I < nc; ++I) {  // R = P^T: the fine nodes that interpolate from I
        const int fc = fpos[I];
        for (int q = 0; q < 3; ++q) ri[3 * I + q] = fc;
        rw[3 * I + 1] = 1.0;
        if (fc - 1 >= 0 && !is_c[s][fc - 1]) {
          ri[3 * I] = fc - 1;
          rw[3 * I] = pw[2 * (fc - 1) + 1];  // fine fc - 1: its right coarse neighbour is I
        }
        if (fc + 1 < nf && !is_c[s][fc + 1]) {
          ri[3 * I + 2] = fc + 1;
          rw[3 * I + 2] = pw[2 * (fc + 1)];  // fine fc + 1: its left coarse neighbour is I
        }
      }
      if (int e = mg_upload(c, L, pi, &x.pi[s])) return e;
      if (int e = mg_upload(c, L, pw, &x.pw[s])) return e;
      if (int e = mg_upload(c, L, ri, &x.ri[s])) return e;
      if (int e = mg_upload(c, L, rw, &x.rw[s])) return e;
      x.fn[s] = nf;
      x.cn[s] = nc;
      x.coarse[s] = coarsen[s] ? 1 : 0;
    }
    x.f_kb = 0;
    x.f_ke = x.fn[2];
    x.c_kb = 0;
    x.c_ke = x.cn[2];
    for (int s = 0; s < 3; ++s) Xp[s] = L.X[s];
  }
  c->mg_on = true;
  return TV_OK;
}

// per Newton iteration: T injected down the hierarchy (DG: the vertex mean of
// the cell-local values onto the CG level), coarse Jacobi diagonals
static bool mg_prep_split();

static void mg_prepare(Ctx* c, const double* T) {
  // after the first call (dinv interiors in place): the CG levels below the
  // base in two launches (launch_mg_prepare)
  const size_t base = c->mg_dg ? 1 : 0;  // DG: level 1 is the vertex mean of the DG field
  const size_t ncg = c->mg.size() - std::min(c->mg.size(), base);
  bool ready = ncg > 0 && ncg <= (size_t)kMgPrepMax && !mg_prep_split();
  for (size_t l = base; l < c->mg.size() && ready; ++l)
    ready = c->mg[l].dinv_interior && cg_uses_march(c->mg[l].g) && c->mg[l].g.bnodes != nullptr;
  if (ready) {
    if (base == 1) {
      MgLevel& L = c->mg[0];
      launch_mg_dg_T(c->dg.c0, c->dg.c1, c->dg.c2, T, L.T, c->stream);
      if (c->dggface) launch_dg_gface(c->dg, T, c->dggface, c->stream);
      launch_cg_diag(L.g, L.T, L.dinv, 1, c->stream, true);
    }
    MgPrep p{};
    p.nlev = (int)ncg;
    p.Tbase = base == 1 ? c->mg[0].T : T;
    for (size_t i = 0; i < ncg; ++i) {
      MgLevel& L = c->mg[base + i];
      p.xf[i] = L.xf;
      p.T[i] = L.T;
      p.dinv[i] = L.dinv;
      p.g[i] = L.g;
      p.off_n[i + 1] = p.off_n[i] + (L.n + 63) / 64 * 64;
      p.off_b[i + 1] = p.off_b[i] + (L.g.n_bnodes + 63) / 64 * 64;
    }
    launch_mg_prepare(p, c->stream);
    return;
  }
  const double* Tf = T;
  for (size_t l = 0; l < c->mg.size(); ++l) {
    MgLevel& L = c->mg[l];
    if (l == 0 && c->mg_dg) {
      launch_mg_dg_T(c->dg.c0, c->dg.c1, c->dg.c2, T, L.T, c->stream);
      if (c->dggface) launch_dg_gface(c->dg, T, c->dggface, c->stream);
    }
    else launch_mg_inject(L.xf, Tf, L.T, c->stream);
    launch_cg_diag(L.g, L.T, L.dinv, 1, c->stream, L.dinv_interior);
    L.dinv_interior = true;
    Tf = L.T;
  }
}

// V-cycle on coarse level l >= 1 (index l - 1 in c->mg): rhs b -> x; the
// pre-smoothing step from 0 (x = omega D^-1 b) was formed by the restriction
// that produced b.  The J x before the restriction is complete (k_cg_addfaces:
// a per-node facet term inside the 27-point gather measured slower); the one
// before the post-smoothing leaves the facet terms of the faces along the
// march to that pointwise consumer (FaceAdd).
// The prolongation from coarse level index ci (c->mg[ci]) into its finer level:
// where that level has a post-smoothing step (not the coarsest) and the
// 2 x 2 block prolongation runs, the step is applied on the fly (CoarsePost)
// and mg_level skipped its k_mg_jacobi launch.
static void mg_prolong_from(Ctx* c, size_t ci, double* xf, const double* mask) {
  MgLevel& C = c->mg[ci];
  const bool smoothed = ci + 1 < c->mg.size() && mg_prolong_smooths(C.xf);
  if (smoothed) {
    const CoarsePost cp{C.b, C.w, C.dinv, C.omega, cg_face_add(C.g, 0)};
    launch_mg_prolong(C.xf, c->st, xf, C.x, mask, c->stream, &cp);
  } else {
    launch_mg_prolong(C.xf, c->st, xf, C.x, mask, c->stream);
  }
}

static void mg_level(Ctx* c, size_t l) {
  MgLevel& L = c->mg[l - 1];
  hipStream_t s = c->stream;
  if (l < c->mg.size()) {
    const MgLevel& C = c->mg[l];
    const FaceAdd fa = cg_face_add(L.g, 0);
    if (fa.on && mg_restrict_folds_faces(C.xf)) {  // the restriction adds the facet terms (no k_cg_addfaces)
      launch_cg_japply_partial(L.g, L.T, L.x, L.w, c->st, s);
      launch_mg_restrict(C.xf, c->st, L.b, L.w, &fa, nullptr, C.b, C.dinv, C.omega, C.x, s);
    } else {
      launch_cg_japply(L.g, L.T, L.x, L.w, nullptr, nullptr, s, c->st);
      launch_mg_restrict(C.xf, c->st, L.b, L.w, nullptr, nullptr, C.b, C.dinv, C.omega, C.x, s);
    }
    mg_level(c, l + 1);
    mg_prolong_from(c, l, L.x, nullptr);
    launch_cg_japply_partial(L.g, L.T, L.x, L.w, c->st, s);
    // post-smoothing, unless the prolongation out of this level applies it (mg_prolong_from)
    if (!mg_prolong_smooths(L.xf))
      launch_mg_jacobi(L.n, c->st, L.b, L.w, &fa, L.dinv, L.omega, L.x, 1, s);
  }
}

// TVFEM_MG_PREP=split (with TVFEM_EXPERIMENTS=1): the per-level injection and
// boundary-diagonal launches instead of the two merged ones
static bool mg_prep_split() {
  static const bool on = [] {
    const char* v = experiment_env("TVFEM_MG_PREP");
    return v != nullptr && v[0] == 's';
  }();
  return on;
}

// TVFEM_MG_FOLD0=1 (with TVFEM_EXPERIMENTS=1): level 0's facet terms added by the
// restriction too, as on the coarse levels (instead of k_cg_addfaces)
static bool mg_fold0() {
  static const bool on = [] {
    const char* v = experiment_env("TVFEM_MG_FOLD0");
    return v != nullptr && v[0] == '1';
  }();
  return on;
}

// TVFEM_MG_POST=split (with TVFEM_EXPERIMENTS=1): level 0's last J x and the
// post-smoothing as two launches (k_cg_march + k_mg_post) instead of the fused march
static bool mg_post_split() {
  static const bool on = [] {
    const char* v = experiment_env("TVFEM_MG_POST");
    return v != nullptr && v[0] == 's';
  }();
  return on;
}

// level 0: x0 = omega dinv r is in c->mgx (k_mg_update); coarse correction,
// post-smoothing into z with the (z.z, z.r) reduction tail
static int mg_apply0(Ctx* c, const double* T, const RedTail* tail) {
  const int64_t n = c->nT;
  hipStream_t s = c->stream;
  const double* mask = c->dir_on ? c->dinv : nullptr;  // Dirichlet: the free subspace
  if (c->mg_dg) {  // DG1 level 0: complete DG J x (Robin facets inline), vertex sums / injection to CG1
    const DgGrid& d = c->dg;
    MgLevel& C = c->mg[0];
    launch_dg_japply(d, T, c->mgx, c->w, nullptr, nullptr, s, c->st);
    launch_mg_dg_restrict(d.c0, d.c1, d.c2, c->st, c->r, c->w, mask, C.b, C.dinv, C.omega, C.x, s);
    mg_level(c, 1);
    launch_mg_dg_prolong(d.c0, d.c1, d.c2, c->st, c->mgx, C.x, mask, s);
    launch_dg_japply(d, T, c->mgx, c->w, nullptr, nullptr, s, c->st);
    if (c->dggface)
      return launch_dg_bpost(d, c->st, c->mgx, c->r, c->w, c->dggface, c->mg_omega0, c->z, c->partials, tail, s);
    return launch_mg_post(n, c->st, c->mgx, c->r, c->w, nullptr, c->dinv, c->mg_omega0, c->z, c->partials, tail, s);
  }
  const FaceAdd fa = cg_face_add(c->cg, 0);
  if (!c->mg.empty()) {
    MgLevel& C = c->mg[0];
    if (mg_fold0() && fa.on && mg_restrict_folds_faces(C.xf)) {
      launch_cg_japply_partial(c->cg, T, c->mgx, c->w, c->st, s);
      launch_mg_restrict(C.xf, c->st, c->r, c->w, &fa, mask, C.b, C.dinv, C.omega, C.x, s);
    } else {
      launch_cg_japply(c->cg, T, c->mgx, c->w, nullptr, nullptr, s, c->st);
      launch_mg_restrict(C.xf, c->st, c->r, c->w, nullptr, mask, C.b, C.dinv, C.omega, C.x, s);
    }
    mg_level(c, 1);
    mg_prolong_from(c, 0, c->mgx, mask);
  }
  // J x, post-smoothing and (z.z, z.r) in the march epilogue (+ the side-face pass)
  if (!mg_post_split()) {
    const int nrec = launch_cg_japply_post(c->cg, T, c->mgx, c->r, c->dinv, c->mg_omega0, c->z, c->st, c->partials,
                                           tail, s);
    if (nrec >= 0) return nrec;
  }
  launch_cg_japply_partial(c->cg, T, c->mgx, c->w, c->st, s);
  return launch_mg_post(n, c->st, c->mgx, c->r, c->w, &fa, c->dinv, c->mg_omega0, c->z, c->partials, tail, s);
}

static int mg_iteration(Ctx* c, const double* T, int it) {
  const int64_t n = c->nT;
  const int slot = c->ts_next + it;
  uint64_t* ts = (c->ktime && (it % c->kstride) == 0 && slot < kTsCap) ? c->d_ts + 4 * slot : nullptr;
  RedTail t1{c->counters, c->partials, c->sums, c->st, 2, ts};
  int np = 0;
  if (!op_japply_fused(c, T, &np, &t1, it))  // p <- z + b p ; w <- J p ; p.w ; alpha
    if (int e = reduce_logic(c, np, 1, 2, 1)) return e;
  const FaceAdd fa = c->mg_dg ? FaceAdd{} : cg_face_add(c->cg, 0);  // DG: w is complete
  if (c->dggface)
    launch_dg_bupdate(c->dg, c->st, c->pA, c->pB, c->w, c->dggface, c->mg_omega0, c->r, c->f[TV_F_DX].ptr, c->mgx, it, 0,
                      c->stream);
  else
    launch_mg_update(n, c->st, c->pA, c->pB, c->w, &fa, c->dinv, c->mg_omega0, c->r, c->f[TV_F_DX].ptr, c->mgx, it, 0,
                     c->stream);
  RedTail t2{c->counters + kTailCounters, c->partials, c->sums, c->st, 3, nullptr};
  mg_apply0(c, T, &t2);  // z <- V(r); z.z, z.r; beta, convergence
  return TV_OK;
}

static int pcg_solve_mg(Ctx* c, const double* T, int* its, int* reason) {
  const int64_t n = c->nT;
  PcgState h{};
  h.rtol = c->O.ksp_rtol;
  h.atol = c->O.ksp_atol;
  h.dtol = c->O.ksp_dtol;
  h.max_it = c->O.ksp_max_it;
  // from pinned memory (an asynchronous upload; a pageable source is staged by
  // the runtime -- no step-time change measured at C2 / C3 / C4)
  c->h_st[2] = h;
  HIPC(hipMemcpyAsync(c->st, &c->h_st[2], sizeof(PcgState), hipMemcpyHostToDevice, c->stream));
  mg_prepare(c, T);
  if (c->dggface)
    launch_dg_bupdate(c->dg, c->st, c->pA, c->pB, c->w, c->dggface, c->mg_omega0, c->r, c->f[TV_F_DX].ptr, c->mgx, 0, 1,
                      c->stream);  // dx <- 0, x0 <- omega B^-1 r
  else
    launch_mg_update(n, c->st, c->pA, c->pB, c->w, nullptr, c->dinv, c->mg_omega0, c->r, c->f[TV_F_DX].ptr, c->mgx, 0, 1,
                     c->stream);  // dx <- 0, x0 <- omega dinv r
  RedTail t0{c->counters + kTailCounters, c->partials, c->sums, c->st, 1, nullptr};
  mg_apply0(c, T, &t0);  // z <- V(r); dp, beta (KSPCG init)
  if (c->ktime && c->ts_next + c->O.ksp_max_it + 8 > kTsCap)
    if (int e = ts_flush(c)) return e;
  // an MG iteration is ~25 launches: the previous solve's count (hint) is queued
  // right behind the init, with no host wait in between (the GPU would idle
  // while the host enqueues ~100 launches; an init that already converged
  // makes every queued launch exit at once), then one iteration at a time
  // behind a poll.  The Newton solves of a step take near-constant counts, so
  // the hint usually ends the solve at the first poll.
  int launched = 0;
  auto enqueue = [&](int nb) -> int {
    for (int b = 0; b < nb; ++b)
      if (int e = mg_iteration(c, T, launched + b)) return e;
    launched += nb;
    HIPC(hipGetLastError());
    HIPC(hipMemcpyAsync(&c->h_st[0], c->st, sizeof(PcgState), hipMemcpyDeviceToHost, c->stream));
    HIPC(hipEventRecord(c->evp[0], c->stream));
    return TV_OK;
  };
  if (int e = enqueue(std::max(1, c->pcg_hint))) return e;
  for (;;) {
    HIPC(hipEventSynchronize(c->evp[0]));
    if (c->h_st[0].done) break;
    if (launched > c->O.ksp_max_it + 2) return c->fail(TV_ERR_KSP, "PCG: iteration guard exceeded");
    if (int e = enqueue(1)) return e;
  }
  *its = c->h_st[0].it;
  *reason = c->h_st[0].reason;
  // level 0 updates dx in pairs of iterations from iteration 1 on (k_mg_update /
  // k_dg_bupdate DXU): solves of 0 / 1 iterations and the last step of an odd-length one
  launch_mg_dx_finish(n, c->st, c->pA, c->pB, c->f[TV_F_DX].ptr, *its, c->stream);
  c->pcg_hint = std::max(1, c->h_st[0].it);
  if (c->ktime) {
    for (int it = 0; it < *its; it += c->kstride)
      if (c->ts_next + it < kTsCap) c->ts_pending.push_back(c->ts_next + it);
    c->ts_next = std::min(kTsCap, c->ts_next + launched);
  }
  return TV_OK;
}

// ---- single-reduction PCG (Chronopoulos-Gear form, k_cgs_march) -------------
// w of the owned boundary planes + the face-workgroup facet terms (the value a
// neighbour's ghost plane must hold), packed for the halo
__global__ __launch_bounds__(kBlock) void k_cgs_pack(CgGrid g, const double* __restrict__ w,
                                                     const double* __restrict__ ff, int raxis,
                                                     double* __restrict__ out) {
  const int64_t plane = (int64_t)g.n0 * g.n1;
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < 2 * plane; t += (int64_t)gridDim.x * kBlock) {
    const int side = (int)(t / plane);
    const int64_t e = t - side * plane;
    const int k = side ? g.k_end - 1 : g.k_begin;
    const int i = (int)(e % g.n0), j = (int)(e / g.n0);
    // facet terms in the order of k_cgs_march: x face, then the row-axis face
    double fx = 0.0, fr = 0.0;
    const int fxi = (i == 0) ? 0 : (i == g.n0 - 1 ? 1 : -1);
    if (fxi >= 0 && g.ffoff[fxi] >= 0) fx = ff[g.ffoff[fxi] + j + (int64_t)g.n1 * k];
    const int c = (raxis == 1) ? j : k, n = (raxis == 1) ? g.n1 : g.n2;
    const int sd = (c == 0) ? 0 : (c == n - 1 ? 1 : -1);
    if (sd >= 0 && g.ffoff[2 * raxis + sd] >= 0) fr = ff[g.ffoff[2 * raxis + sd] + i + (int64_t)g.n0 * ((raxis == 1) ? k : j)];
    out[t] = w[e + plane * k] + (fx + fr);
  }
}

static int cgs_raxis(const Ctx* c) { return (c->cg.n2 >= c->cg.n1) ? 2 : 1; }  // = plan(g).raxis

// ghost planes of w_i: neighbours' packed boundary planes (RCCL group with
// the all-reduce of the iteration's sums, or the host-staged transport)
static int cgs_exchange(Ctx* c, double* wout, const double* fout) {
  const CgGrid& g = c->cg;
  const int64_t plane = (int64_t)g.n0 * g.n1;
  const int blocks = (int)std::min<int64_t>(1024, (2 * plane + kBlock - 1) / kBlock);
  hipLaunchKernelGGL(k_cgs_pack, dim3(blocks), dim3(kBlock), 0, c->stream, g, wout, fout, cgs_raxis(c), c->wsend);
  if (c->host_sendrecv) {
    if (int e = allreduce(c, c->sums, 3)) return e;
    double* s_lo = c->h_halo;
    double* s_hi = c->h_halo + plane;
    double* r_lo = c->h_halo + 2 * plane;
    double* r_hi = c->h_halo + 3 * plane;
    HIPC(hipMemcpyAsync(s_lo, c->wsend, 2 * plane * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPC(hipStreamSynchronize(c->stream));
    if (g.g_lo && c->host_sendrecv(s_lo, (size_t)plane, c->rank - 1, r_lo, (size_t)plane, c->rank - 1, c->host_user))
      return c->fail(TV_ERR_COMM, "host sendrecv failed");
    if (g.g_hi && c->host_sendrecv(s_hi, (size_t)plane, c->rank + 1, r_hi, (size_t)plane, c->rank + 1, c->host_user))
      return c->fail(TV_ERR_COMM, "host sendrecv failed");
    if (g.g_lo) HIPC(hipMemcpyAsync(wout, r_lo, plane * sizeof(double), hipMemcpyHostToDevice, c->stream));
    if (g.g_hi) HIPC(hipMemcpyAsync(wout + plane * g.k_end, r_hi, plane * sizeof(double), hipMemcpyHostToDevice, c->stream));
    return TV_OK;
  }
  // one group: the 3-scalar all-reduce and the ghost planes of w (<= 2 peers)
  NCCLC(ncclGroupStart());
  NCCLC(ncclAllReduce(c->sums, c->sums, 3, ncclDouble, ncclSum, c->comm, c->stream));
  if (g.g_lo) {
    NCCLC(ncclSend(c->wsend, plane, ncclDouble, c->rank - 1, c->comm, c->stream));
    NCCLC(ncclRecv(wout, plane, ncclDouble, c->rank - 1, c->comm, c->stream));
  }
  if (g.g_hi) {
    NCCLC(ncclSend(c->wsend + plane, plane, ncclDouble, c->rank + 1, c->comm, c->stream));
    NCCLC(ncclRecv(wout + plane * g.k_end, plane, ncclDouble, c->rank + 1, c->comm, c->stream));
  }
  NCCLC(ncclGroupEnd());
  return TV_OK;
}

static CgsBuffers cgs_buffers(Ctx* c, const double* T, int it) {
  // iteration it reads parity (it - 1) & 1 and writes it & 1; r_0 is the Newton
  // residual (c->r), read by iterations 0 and 1
  CgsBuffers v{};
  const int o = (it + 1) & 1, w = it & 1;
  double* W[2] = {c->w, c->cw1};
  v.T = T;
  v.rin = (it <= 1) ? c->r : c->cr[o];
  v.rout = c->cr[w];
  v.sin = c->cs[o];
  v.sout = c->cs[w];
  v.win = W[o];
  v.wout = W[w];
  v.fin = c->cg.ffbuf[o];
  v.fout = c->cg.ffbuf[w];
  v.p = c->pA;
  v.x = c->f[TV_F_DX].ptr;
  v.dinv = c->dinv;
  return v;
}

static int cgs_iteration(Ctx* c, const double* T, int it) {
  const bool multi = multi_rank(c);
  const int slot = c->ts_next + it;
  uint64_t* ts = (c->ktime && (it % c->kstride) == 0 && slot < kTsCap) ? c->d_ts + 4 * slot : nullptr;
  const int kind = multi ? 0 : (it == 0 ? 4 : 5);
  RedTail rt{c->counters, c->partials, c->sums, c->st, kind, ts};
  const CgsBuffers v = cgs_buffers(c, T, it);
  launch_cg_cgs(c->cg, it == 0, v, c->st, c->partials, c->stream, &rt, it, (multi && it > 0) ? c->sums : nullptr);
  if (multi)
    if (int e = cgs_exchange(c, v.wout, v.fout)) return e;
  return TV_OK;
}

static int pcg_solve_cgs(Ctx* c, const double* T, int* its, int* reason) {
  PcgState h{};
  h.rtol = c->O.ksp_rtol;
  h.atol = c->O.ksp_atol;
  h.dtol = c->O.ksp_dtol;
  h.max_it = c->O.ksp_max_it;
  // from pinned memory (an asynchronous upload; a pageable source is staged by
  // the runtime -- no step-time change measured at C2 / C3 / C4)
  c->h_st[2] = h;
  HIPC(hipMemcpyAsync(c->st, &c->h_st[2], sizeof(PcgState), hipMemcpyHostToDevice, c->stream));
  // ghost planes of r_0 and diag^-1 (the halo rows recompute z there)
  if (int e = halo(c, c->r)) return e;
  if (int e = halo(c, c->dinv)) return e;
  if (c->ktime && c->ts_next + c->O.ksp_max_it + 4 * c->O.pcg_batch + 8 > kTsCap)
    if (int e = ts_flush(c)) return e;
  int launched = 0, slot = 0;
  auto enqueue = [&](int nb, int k) -> int {
    for (int b = 0; b < nb; ++b)
      if (int e = cgs_iteration(c, T, launched + b)) return e;
    launched += nb;
    HIPC(hipGetLastError());
    HIPC(hipMemcpyAsync(&c->h_st[k], c->st, sizeof(PcgState), hipMemcpyDeviceToHost, c->stream));
    HIPC(hipEventRecord(c->evp[k], c->stream));
    return TV_OK;
  };
  // iteration 0 and the first batch, then one more iteration queued behind
  // every poll (see pcg_solve); multi-rank the state lags one launch
  const int lag = multi_rank(c) ? 1 : 0;
  const int small = 1 + lag;
  if (int e = enqueue(1 + std::max(1, c->pcg_hint > 4 ? c->pcg_hint - 3 : c->O.pcg_batch), 0)) return e;
  for (;;) {
    if (int e = enqueue(small, slot ^ 1)) return e;
    HIPC(hipEventSynchronize(c->evp[slot]));
    if (c->h_st[slot].done) break;
    if (launched > c->O.ksp_max_it + 2 * small + 4) return c->fail(TV_ERR_KSP, "PCG: iteration guard exceeded");
    slot ^= 1;
  }
  *its = c->h_st[slot].it;
  *reason = c->h_st[slot].reason;
  c->pcg_hint = *its;
  if (c->ktime) {
    for (int it = 1; it <= *its; it += c->kstride)  // productive iterations (iteration 0 is the init launch)
      if (c->ts_next + it < kTsCap) c->ts_pending.push_back(c->ts_next + it);
    c->ts_next = std::min(kTsCap, c->ts_next + launched);
  }
  return TV_OK;
}

static const char* reason_str(int r) {
  switch (r) {
    case R_DIV_ITS: return "DIVERGED_ITS";
    case R_DIV_DTOL: return "DIVERGED_DTOL";
    case R_DIV_INDEF_PC: return "DIVERGED_INDEFINITE_PC";
    case R_DIV_NANINF: return "DIVERGED_NANORINF";
    case R_DIV_INDEF_MAT: return "DIVERGED_INDEFINITE_MAT";
    default: return "UNKNOWN";
  }
}

// ---- Dirichlet mode ----------------------------------------------------------
struct BndTest {
  CgGrid g;
  const unsigned char* mask;  // unstructured: boundary vertices (else nullptr)
};
__device__ __forceinline__ bool cg_on_boundary(const CgGrid& g, int64_t n);
__device__ __forceinline__ bool on_boundary(const BndTest& b, int64_t n) {
  return b.mask ? b.mask[n] != 0 : cg_on_boundary(b.g, n);
}
__device__ __forceinline__ bool cg_on_boundary(const CgGrid& g, int64_t n) {
  const int64_t plane = (int64_t)g.n0 * g.n1;
  const int k = (int)(n / plane);
  const int64_t rem = n - (int64_t)k * plane;
  const int j = (int)(rem / g.n0), i = (int)(rem - (int64_t)j * g.n0);
  return (i == 0 && g.bnd[0][0]) || (i == g.n0 - 1 && g.bnd[0][1]) || (j == 0 && g.bnd[1][0]) ||
         (j == g.n1 - 1 && g.bnd[1][1]) || (k == 0 && g.bnd[2][0]) || (k == g.n2 - 1 && g.bnd[2][1]);
}
// dB = T - value on constrained nodes, 0 elsewhere (every local node)
__global__ __launch_bounds__(kBlock) void k_bc_dvec(BndTest b, const double* __restrict__ T, double value,
                                                    double* __restrict__ dB, int64_t n) {
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < n; t += (int64_t)gridDim.x * kBlock)
    dB[t] = on_boundary(b, t) ? T[t] - value : 0.0;
}
// F -= J dB (lifting; the constrained rows are never read: diag^-1 = 0 there)
// and diag^-1 = 0 on constrained nodes, so z = B r and every Krylov vector
// stay in the free subspace: PCG on P J P with the Jacobi preconditioner P B P
// read-only sweep (cache state for the flushed timing of tv_time_kernel id 10):
// one sum per workgroup into out[block] so the loads are not dead
__global__ __launch_bounds__(kBlock) void k_read_sweep(const double* __restrict__ a, int64_t n, double* out) {
  double acc = 0.0;
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < n; t += (int64_t)gridDim.x * kBlock) acc += a[t];
  if (acc == 12345.678) out[blockIdx.x] = acc;  // practically never: keeps the loads
}

__global__ __launch_bounds__(kBlock) void k_bc_lift(BndTest b, double* __restrict__ F, const double* __restrict__ JdB,
                                                    double* __restrict__ dinv, int64_t n) {
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < n; t += (int64_t)gridDim.x * kBlock) {
    F[t] -= JdB[t];
    if (on_boundary(b, t)) dinv[t] = 0.0;
  }
}
// dx += dB (the constrained part of the Newton step: x - dx lands on the value)
__global__ __launch_bounds__(kBlock) void k_bc_step(double* __restrict__ dx, const double* __restrict__ dB, int64_t n) {
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < n; t += (int64_t)gridDim.x * kBlock) dx[t] += dB[t];
}

static int dirichlet_pre(Ctx* c, const double* T) {
  const int64_t n = c->nT;
  const int blocks = (int)std::min<int64_t>(4096, (n + kBlock - 1) / kBlock);
  const BndTest bt{c->cg, c->um ? c->um_bmask : nullptr};
  hipLaunchKernelGGL(k_bc_dvec, dim3(blocks), dim3(kBlock), 0, c->stream, bt, T, c->dir_value, c->dB, n);
  op_japply(c, T, c->dB, c->dtmp, nullptr, nullptr);
  hipLaunchKernelGGL(k_bc_lift, dim3(blocks), dim3(kBlock), 0, c->stream, bt, c->r, c->dtmp, c->dinv, n);
  HIPC(hipGetLastError());
  return TV_OK;
}

// dolfinx NewtonSolver::solve, convergence_criterion = "incremental"
static int newton(Ctx* c, int* out_its, int* out_kits, int* out_conv) {
  double* T = c->f[TV_F_T].ptr;
  const double* Tp = c->f[TV_F_T_PREV].ptr;
  // NonlinearProblem.form: ghost update of the state before the first F
  // (ThermoViscoProblem.py:351 scatter_forward); every rank enters it, every step
  if (int e = halo(c, T)) return e;
  if (int e = halo(c, c->f[TV_F_T_PREV].ptr)) return e;
  const int64_t off = c->ownT_off, n = c->ownT_n;
  int its = 0, kits = 0;
  bool conv = false;
  double r0 = 0.0, rn = 0.0;
  // F(u); on the CG march path the residual's boundary pass also rewrites the
  // boundary rows of dinv for the same u once the interior is in place
  auto residual = [&]() -> bool {
    if (!c->um && c->fam_T == TV_CG && c->dinv_interior)
      if (launch_cg_residual_diag(c->cg, T, Tp, c->r, c->dinv, c->stream)) return true;
    op_residual(c, T, Tp, c->r);
    return false;
  };
  bool dinv_fresh = residual();
  while (!conv && its < c->O.newton_max_it) {
    if (!c->dggface) {  // J(u) (matrix-free) + Jacobi PC setup (DG GMG: cell blocks)
      if (!c->um && c->fam_T == TV_CG) {
        // the T-independent interior of dinv is written once; then the boundary nodes only
        if (!dinv_fresh) launch_cg_diag(c->cg, T, c->dinv, 1, c->stream, c->dinv_interior);
        c->dinv_interior = true;
      } else {
        op_diag(c, T, c->dinv, 1);
      }
    }
    dinv_fresh = false;
    const bool dir = c->dir_on && c->fam_T == TV_CG;
    if (dir)
      if (int e = dirichlet_pre(c, T)) return e;
    int k = 0, reason = 0;
    if (int e = (c->mg_on ? pcg_solve_mg(c, T, &k, &reason)
                          : (c->cgs ? pcg_solve_cgs(c, T, &k, &reason) : pcg_solve(c, T, &k, &reason))))
      return e;
    kits += k;
    if (reason < 0)
      return c->fail(TV_ERR_KSP, std::string("Krylov solver did not converge (") + reason_str(reason) + ")");
    if (dir)
      hipLaunchKernelGGL(k_bc_step, dim3((int)std::min<int64_t>(4096, (c->nT + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                         c->stream, c->f[TV_F_DX].ptr, c->dB, c->nT);
    // u <- u - dx; ||dx||^2 by a separate one-block reduce (a reduction tail on
    // the update's 1024 workgroups measured 7 us slower: 1024 serialised arrivals)
    launch_newton_update(n, T + off, c->f[TV_F_DX].ptr + off, c->partials, c->stream);
    if (int e = reduce_logic(c, pcg_vec_blocks(n), 1, 0, 0)) return e;
    HIPC(hipMemcpyAsync(c->h_sums, c->sums, sizeof(double), hipMemcpyDeviceToHost, c->stream));
    if (int e = halo(c, T)) return e;
    HIPC(hipStreamSynchronize(c->stream));
    rn = std::sqrt(c->h_sums[0]);
    ++its;
    if (its == 1) {
      r0 = rn;  // residual0 = ||dx_1||; no test at the first iteration
      conv = false;
    } else {
      const double rel = rn / r0;
      conv = (rel < c->O.newton_rtol) || (rn < c->O.newton_atol);
    }
    // dolfinx assembles F after every update; in the incremental criterion that
    // last F is never read, so it is assembled only when another iteration follows.
    if (!conv && its < c->O.newton_max_it) dinv_fresh = residual();
  }
  HIPC(hipGetLastError());
  c->last_newton = its;
  c->last_krylov = kits;
  c->last_dx = rn;
  if (out_its) *out_its = its;
  if (out_kits) *out_kits = kits;
  if (out_conv) *out_conv = conv ? 1 : 0;
  if (!conv && c->O.error_on_nonconvergence)
    return c->fail(TV_ERR_NOT_CONVERGED, "Newton solver did not converge because maximum number of iterations reached");
  return TV_OK;
}

// --------------------------------------------------------------------------------------
// viscoelastic update
// --------------------------------------------------------------------------------------
static void visco_setup(Ctx* c, ViscoConst& k, ViscoFields& v) {
  const tv_params& P = c->P;
  k.H_over_Rg = P.H / P.Rg;
  k.inv_Tb = 1.0 / P.Tb;
  k.dt = P.dt;
  k.half_dt = P.dt / 2;
  k.alpha_s = P.alpha_solid;
  k.dalpha = P.alpha_liquid - P.alpha_solid;
  k.inv_dim = 1.0 / c->dim;
  k.chi = 0.5;  // ViscoelasticModel.py:15
  k.paper = (c->O.model_mode == TV_MODEL_PAPER) ? 1 : 0;
  for (int i = 0; i < 6; ++i) {
    k.lambda_m[i] = P.lambda_m[i]; k.m_n[i] = P.m_n[i];
    k.lambda_g[i] = P.lambda_g[i]; k.g_n[i] = P.g_n[i];
    k.lambda_k[i] = P.lambda_k[i]; k.k_n[i] = P.k_n[i];
  }
  std::memset(&v, 0, sizeof(v));
  v.sT = c->nT;
  v.sS = c->nS;
  v.T = c->f[TV_F_T].ptr; v.Tp = c->f[TV_F_T_PREV].ptr; v.Tn = c->f[TV_F_T_NEXT].ptr;
  v.phi = c->f[TV_F_PHI].ptr; v.phin = c->f[TV_F_PHI_NEXT].ptr; v.xi = c->f[TV_F_XI].ptr;
  v.Tf = c->f[TV_F_TF].ptr; v.Tfp = c->f[TV_F_TF_PARTIAL].ptr;
  v.th = c->f[TV_F_THERMAL_STRAIN].ptr; v.tot = c->f[TV_F_TOTAL_STRAIN].ptr; v.dev = c->f[TV_F_DEVIATORIC_STRAIN].ptr;
  v.ds = c->f[TV_F_DS_PARTIAL].ptr; v.dsig = c->f[TV_F_DSIGMA_PARTIAL].ptr;
  v.st = c->f[TV_F_S_TILDE].ptr; v.sgt = c->f[TV_F_SIGMA_TILDE].ptr;
  v.sp = c->f[TV_F_S_PARTIAL].ptr; v.sgp = c->f[TV_F_SIGMA_PARTIAL].ptr;
  v.sigma = c->f[TV_F_SIGMA].ptr;
  v.tflag = c->tflag;
  v.Tfo = c->Tfo;
}

static int visco(Ctx* c, bool copy_Tprev) {
  ViscoConst k;
  ViscoFields v;
  visco_setup(c, k, v);
  const int all = c->O.materialize ? 1 : 0;
  if (c->fam_T == c->fam_S) {
    v.n = c->ownT_n;
    v.off_T = c->ownT_off;
    v.off_S = c->ownS_off;
    v.copy_Tprev = copy_Tprev ? 1 : 0;
    launch_visco(c->dim, all, k, v, c->stream);
    if (copy_Tprev && c->ownT_off > 0) {  // ghost planes of T_prev
      launch_copy(v.Tp, v.T, c->ownT_off, c->stream);
    }
    if (copy_Tprev && c->nT > c->ownT_off + c->ownT_n) {
      const int64_t o = c->ownT_off + c->ownT_n;
      launch_copy(v.Tp + o, v.T + o, c->nT - o, c->stream);
    }
  } else {
    v.n = c->ownT_n;
    v.off_T = c->ownT_off;
    launch_visco_Tpass(c->dim, all, k, v, c->stream);
    v.n = c->ownS_n;
    v.off_S = c->ownS_off;
    v.map = c->map;
    launch_visco_Spass(c->dim, all, k, v, c->stream);
    if (copy_Tprev) launch_copy(v.Tp, v.T, c->nT, c->stream);
  }
  HIPC(hipGetLastError());
  return TV_OK;
}

}  // namespace tv

using namespace tv;

// ======================================================================================
// C-ABI
// ======================================================================================
extern "C" {

int tv_abi_version(void) { return TV_ABI_VERSION; }

const char* tv_last_error(const void* ctx) {
  if (ctx) return static_cast<const Ctx*>(ctx)->err.c_str();
  std::lock_guard<std::mutex> lk(g_err_mu);
  return g_err.c_str();
}

void tv_default_options(tv_options* o) {
  o->newton_rtol = 1e-12;  // ThermoViscoProblem.py:336
  o->newton_atol = 1e-10;  // dolfinx NewtonSolver default
  o->newton_max_it = 50;   // dolfinx default
  o->error_on_nonconvergence = 1;
  o->ksp_rtol = 1e-5;      // PETSc defaults
  o->ksp_atol = 1e-50;
  o->ksp_dtol = 1e5;
  o->ksp_max_it = 10000;
  o->materialize = 1;
  o->use_graphs = 0;
  o->pcg_batch = 8;
  o->pcg_variant = TV_PCG_AUTO;
  o->model_mode = TV_MODEL_REFERENCE;
  o->preconditioner = TV_PC_JACOBI;
  o->mg_levels = 0;
}

void tv_default_params(tv_params* p) {
  std::memset(p, 0, sizeof(*p));
  // main.py:29-55
  p->f = 0.0; p->epsilon = 0.93; p->sigma = 5.670e-8; p->T_ambient = 600.0; p->T_0 = 800.0;
  p->alpha = 1.0; p->htc = 280.1; p->rho = 2500.0; p->cp = 1433.0; p->k = 1.0;
  p->H = 627.8e3; p->Tb = 869.0; p->Rg = 8.314; p->alpha_solid = 9.10e-6; p->alpha_liquid = 25.10e-6;
  p->Tf_init = 873.0;
  // ViscoelasticModel.py:19-68
  const double m[6] = {5.523e-2, 8.205e-2, 1.215e-1, 2.286e-1, 2.860e-1, 2.265e-1};
  const double lm[6] = {5.965e-4, 1.077e-2, 1.362e-1, 1.505e-1, 6.747e+0, 2.963e+1};
  const double g[6] = {1.585, 2.354, 3.486, 6.558, 8.205, 6.498};
  const double lg[6] = {6.658e-5, 1.197e-3, 1.514e-2, 1.672e-1, 7.497e-1, 3.292e+0};
  const double k[6] = {7.588e-1, 7.650e-1, 9.806e-1, 7.301e+0, 1.347e+1, 1.090e+1};
  const double lk[6] = {5.009e-5, 9.945e-4, 2.022e-3, 1.925e-2, 1.199e-1, 2.033e+0};
  for (int i = 0; i < 6; ++i) {
    p->m_n[i] = m[i]; p->lambda_m[i] = lm[i]; p->g_n[i] = g[i];
    p->lambda_g[i] = lg[i]; p->k_n[i] = k[i]; p->lambda_k[i] = lk[i];
  }
  p->dt = 0.1;  // main.py:16
}

int tv_create(const tv_mesh_desc* mesh, const tv_fe_config* fe, const tv_params* params, const tv_options* opts,
              int device, void** ctx_out) {
  if (!mesh || !fe || !params || !ctx_out) {
    set_global_error("tv_create: null argument");
    return TV_ERR_ARG;
  }
  *ctx_out = nullptr;
  auto c = std::make_unique<Ctx>();
  if (fe->T_degree != 1 || fe->sigma_degree != 1) {
    set_global_error("only degree-1 Lagrange elements are implemented");
    return TV_ERR_ARG;
  }
  if ((fe->T_family != TV_CG && fe->T_family != TV_DG) || (fe->sigma_family != TV_CG && fe->sigma_family != TV_DG)) {
    set_global_error("Only CG and DG elements are supported");
    return TV_ERR_ARG;
  }
  if (!(params->dt > 0.0)) {
    set_global_error("dt must be positive");
    return TV_ERR_ARG;
  }
  c->fam_T = fe->T_family;
  c->fam_S = fe->sigma_family;
  c->P = *params;
  if (opts) c->O = *opts;
  else tv_default_options(&c->O);
  c->device = device;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    set_global_error("no HIP device available: libtvfem requires an MI355X (gfx950) GPU");
    return TV_ERR_HIP;
  }
  if (device < 0 || device >= ndev) {
    set_global_error("device index out of range");
    return TV_ERR_ARG;
  }
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess) {
    set_global_error("HIP stream/event creation failed");
    return TV_ERR_HIP;
  }
  int rc = setup_mesh(c.get(), mesh);
  if (rc == TV_OK) rc = setup_fields(c.get());
  if (rc == TV_OK && c->O.preconditioner == TV_PC_GMG) rc = mg_setup(c.get());
  else if (rc == TV_OK && c->O.preconditioner != TV_PC_JACOBI) rc = c->fail(TV_ERR_ARG, "unknown preconditioner");
  if (rc == TV_OK && hipStreamSynchronize(c->stream) != hipSuccess) rc = c->fail(TV_ERR_HIP, "sync failed");
  if (rc != TV_OK) {
    set_global_error(c->err);
    tv_destroy(c.release());
    return rc;
  }
  *ctx_out = c.release();
  return TV_OK;
}

static int setup_umesh(Ctx* c, const tv_umesh_desc* m) {
  const int d = m->dim;
  if (d != 2 && d != 3) return c->fail(TV_ERR_ARG, "unstructured meshes: dim 2 (quadrilaterals) or 3 (hexahedra)");
  if (c->fam_T != TV_CG || c->fam_S != TV_CG)
    return c->fail(TV_ERR_ARG, "unstructured meshes: CG temperature and stress spaces only");
  if (m->n_vertices < 1 || m->n_cells < 1 || !m->coords || !m->cells) return c->fail(TV_ERR_ARG, "empty mesh");
  if (m->n_vertices >= INT32_MAX) return c->fail(TV_ERR_ARG, "unstructured meshes: < 2^31 vertices");
  const int nl = 1 << d;
  for (int64_t k = 0; k < m->n_cells * nl; ++k)
    if (m->cells[k] < 0 || m->cells[k] >= m->n_vertices) return c->fail(TV_ERR_ARG, "cell vertex index out of range");
  c->um = true;
  c->dim = d;
  c->um_xyz.assign(m->coords, m->coords + 3 * m->n_vertices);
  c->um_cells.assign(m->cells, m->cells + m->n_cells * nl);
  const tv_params& P = c->P;
  UmGrid& g = c->umg;
  g.dt = P.dt; g.dt_alpha = P.dt * P.alpha; g.dt_f = P.dt * P.f;
  g.a_rad = 0.001 * (P.sigma * P.epsilon); g.a_conv = 0.001 * P.htc;
  g.T_amb = P.T_ambient; g.T_amb4 = P.T_ambient * P.T_ambient * P.T_ambient * P.T_ambient;
  std::string err;
  if (um_setup(d, m->n_vertices, m->coords, m->n_cells, m->cells, g, c->umd, c->stream, err) != 0)
    return c->fail(err.rfind("HIP", 0) == 0 ? TV_ERR_HIP : TV_ERR_ARG, err);
  std::vector<unsigned char> bm;
  um_boundary_vertices(c->umd, bm);
  HIPC(hipMalloc(&c->um_bmask, bm.size()));
  HIPC(hipMemcpy(c->um_bmask, bm.data(), bm.size(), hipMemcpyHostToDevice));
  c->nT = c->nS = g.nv;
  c->ownT_off = c->ownS_off = 0;
  c->ownT_n = c->ownS_n = g.nv;
  c->globT_off = c->globS_off = 0;
  return TV_OK;
}

int tv_create_unstructured(const tv_umesh_desc* mesh, const tv_fe_config* fe, const tv_params* params,
                           const tv_options* opts, int device, void** ctx_out) {
  if (!mesh || !fe || !params || !ctx_out) {
    set_global_error("tv_create_unstructured: null argument");
    return TV_ERR_ARG;
  }
  *ctx_out = nullptr;
  auto c = std::make_unique<Ctx>();
  if (fe->T_degree != 1 || fe->sigma_degree != 1) {
    set_global_error("only degree-1 Lagrange elements are implemented");
    return TV_ERR_ARG;
  }
  if (!(params->dt > 0.0)) {
    set_global_error("dt must be positive");
    return TV_ERR_ARG;
  }
  c->fam_T = fe->T_family;
  c->fam_S = fe->sigma_family;
  c->P = *params;
  if (opts) c->O = *opts;
  else tv_default_options(&c->O);
  c->device = device;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    set_global_error("no HIP device available: libtvfem requires an MI355X (gfx950) GPU");
    return TV_ERR_HIP;
  }
  if (device < 0 || device >= ndev) {
    set_global_error("device index out of range");
    return TV_ERR_ARG;
  }
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess) {
    set_global_error("HIP stream/event creation failed");
    return TV_ERR_HIP;
  }
  if (c->O.preconditioner != TV_PC_JACOBI) {
    set_global_error("unstructured meshes: preconditioner TV_PC_JACOBI only");
    return TV_ERR_ARG;
  }
  int rc = setup_umesh(c.get(), mesh);
  if (rc == TV_OK) rc = setup_fields(c.get());
  if (rc == TV_OK && hipStreamSynchronize(c->stream) != hipSuccess) rc = c->fail(TV_ERR_HIP, "sync failed");
  if (rc != TV_OK) {
    set_global_error(c->err);
    tv_destroy(c.release());
    return rc;
  }
  *ctx_out = c.release();
  return TV_OK;
}

int tv_partition_rcb(const tv_umesh_desc* m, int n_parts, int* part_out) {
  if (!m || !part_out || !m->coords || !m->cells || (m->dim != 2 && m->dim != 3)) {
    set_global_error("tv_partition_rcb: bad argument");
    return TV_ERR_ARG;
  }
  std::string err;
  if (um_rcb(m->dim, m->n_vertices, m->coords, m->n_cells, m->cells, n_parts, part_out, err)) {
    set_global_error(err);
    return TV_ERR_ARG;
  }
  return TV_OK;
}

int tv_partition_layout(const tv_mesh_desc* m, int64_t* out) {
  if (!m || !out || m->dim < 1 || m->dim > 3 || m->n_parts < 1 || m->part < 0 || m->part >= m->n_parts) {
    set_global_error("tv_partition_layout: invalid arguments");
    return TV_ERR_ARG;
  }
  int perm[3];
  if (!storage_perm(m, perm)) {
    set_global_error("part_axis must be 1 (y) or 2 (z) for 3D meshes");
    return TV_ERR_ARG;
  }
  int N[3];
  for (int s = 0; s < 3; ++s) N[s] = (perm[s] < 0) ? 1 : m->n_cells[perm[s]] + 1;
  int b0, b1;
  part_planes(N[2], m->n_parts, m->part, &b0, &b1);
  const int64_t plane = (int64_t)N[0] * N[1];
  const int glo = m->part > 0, ghi = m->part < m->n_parts - 1;
  out[0] = perm[0]; out[1] = perm[1]; out[2] = perm[2];
  out[3] = N[0]; out[4] = N[1]; out[5] = N[2];
  out[6] = b0; out[7] = b1;
  out[8] = plane * b0;                          // global offset of the first owned dof
  out[9] = plane * (b1 - b0);                   // owned dofs
  out[10] = plane * ((b1 - b0) + glo + ghi);   // local dofs (owned + ghost planes)
  out[11] = glo; out[12] = ghi;
  return TV_OK;
}

int tv_destroy(void* ctx) {
  if (!ctx) return TV_OK;
  Ctx* c = static_cast<Ctx*>(ctx);
  hipSetDevice(c->device);
  if (c->stream) hipStreamSynchronize(c->stream);
  if (c->out) output_destroy(c->out);
  for (int i = 0; i < TV_NUM_FIELDS; ++i)
    if (c->f[i].alloc && c->f[i].ptr) hipFree(c->f[i].ptr);
  for (double* p : {c->cr[0], c->cr[1], c->cs[0], c->cs[1], c->cw1, c->wsend, c->dB, c->dtmp, c->Tfo})
    if (p) hipFree(p);
  um_free(c->umd);
  if (c->um_bmask) hipFree(c->um_bmask);
  for (MgLevel& L : c->mg) {
    for (void* p : L.bufs) hipFree(p);
    for (int s = 0; s < 3; ++s)
      if (L.coef[s]) hipFree(L.coef[s]);
    if (L.bnodes) hipFree(L.bnodes);
    for (int q = 0; q < 2; ++q)
      if (L.ffbuf[q]) hipFree(L.ffbuf[q]);
  }
  if (c->mgx) hipFree(c->mgx);
  if (c->dggface) hipFree(c->dggface);
  for (double* p : {c->r, c->z, c->pA, c->pB, c->w, c->dinv, c->partials, c->sums, c->scratch})
    if (p) hipFree(p);
  for (int s = 0; s < 3; ++s) {
    if (c->coef[s]) hipFree(c->coef[s]);
    if (c->dgh[s]) hipFree(c->dgh[s]);
  }
  if (c->map) hipFree(c->map);
  if (c->bnodes) hipFree(c->bnodes);
  for (int q = 0; q < 2; ++q)
    if (c->ffbuf[q]) hipFree(c->ffbuf[q]);
  if (c->st) hipFree(c->st);
  if (c->tflag) hipFree(c->tflag);
  if (c->counters) hipFree(c->counters);
  if (c->h_st) hipHostFree(c->h_st);
  if (c->h_sums) hipHostFree(c->h_sums);
  if (c->h_halo) hipHostFree(c->h_halo);
  if (c->comm) ncclCommDestroy(c->comm);
  if (c->ev0) hipEventDestroy(c->ev0);
  if (c->ev1) hipEventDestroy(c->ev1);
  for (int k = 0; k < 2; ++k) {
    if (c->evp[k]) hipEventDestroy(c->evp[k]);
    if (c->vev[k]) hipEventDestroy(c->vev[k]);
  }
  if (c->d_ts) hipFree(c->d_ts);
  if (c->stream) hipStreamDestroy(c->stream);
  delete c;
  return TV_OK;
}

int tv_num_dofs(void* ctx, int space, int64_t* n_owned, int64_t* global_offset) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c) return TV_ERR_ARG;
  if (n_owned) *n_owned = space == 0 ? c->ownT_n : c->ownS_n;
  if (global_offset) *global_offset = space == 0 ? c->globT_off : c->globS_off;
  return TV_OK;
}

int tv_field_block_size(void* ctx, int field, int* bs) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c || field < 0 || field >= TV_NUM_FIELDS) return TV_ERR_ARG;
  const int dd = c->dim * c->dim;
  static const int kind[TV_NUM_FIELDS] = {1, 1, 1, 1, 1, 6, 6, 1, 1, 1, 2, 2, 2, 3, 3, 3, 3, 3, 3, 3, 3, 3, 3, 2, 1, 1};
  const int k = kind[field];
  *bs = (k == 1) ? 1 : (k == 6 ? 6 : (k == 2 ? dd : 6 * dd));
  return TV_OK;
}

int tv_dof_coordinates(void* ctx, int space, double* xyz, size_t n_dofs) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c || !xyz) return TV_ERR_ARG;
  const int fam = space == 0 ? c->fam_T : c->fam_S;
  const int64_t nown = space == 0 ? c->ownT_n : c->ownS_n;
  if ((int64_t)n_dofs != nown) return c->fail(TV_ERR_ARG, "n_dofs mismatch");
  if (c->um) {
    std::memcpy(xyz, c->um_xyz.data(), sizeof(double) * 3 * (size_t)nown);
    return TV_OK;
  }
  std::vector<double> tmp;
  const std::vector<double>* X[3];
  std::vector<double> deg(1, 0.0);
  for (int s = 0; s < 3; ++s) X[s] = (c->perm[s] < 0) ? &deg : &c->coords[c->perm[s]];
  const int N0 = c->Nnode_glob[0], N1 = c->Nnode_glob[1];
  if (fam == TV_CG) {
    const int64_t base = (space == 0 ? c->globT_off : c->globS_off);
    for (int64_t t = 0; t < nown; ++t) {
      const int64_t g = base + t;
      const int ijk[3] = {(int)(g % N0), (int)((g / N0) % N1), (int)(g / ((int64_t)N0 * N1))};
      double p[3] = {0, 0, 0};
      for (int s = 0; s < 3; ++s) if (c->perm[s] >= 0) p[c->perm[s]] = (*X[s])[ijk[s]];
      for (int a = 0; a < 3; ++a) xyz[3 * t + a] = p[a];
    }
  } else {
    const int nl = 1 << c->dim;
    const int C0 = std::max(1, c->Ncell_glob[0]), C1 = std::max(1, c->Ncell_glob[1]);
    const int act[3] = {1, c->perm[1] >= 0, c->perm[2] >= 0};
    for (int64_t t = 0; t < nown; ++t) {
      const int64_t cell = t / nl;
      const int l = (int)(t % nl);
      const int ci[3] = {(int)(cell % C0), (int)((cell / C0) % C1), (int)(cell / ((int64_t)C0 * C1))};
      int bits[3] = {0, 0, 0}, k = 0;
      for (int s = 0; s < 3; ++s) {
        if (!act[s]) continue;
        bits[s] = (l >> k) & 1;
        ++k;
      }
      double p[3] = {0, 0, 0};
      for (int s = 0; s < 3; ++s) if (c->perm[s] >= 0) p[c->perm[s]] = (*X[s])[ci[s] + bits[s]];
      for (int a = 0; a < 3; ++a) xyz[3 * t + a] = p[a];
    }
  }
  return TV_OK;
}

int tv_set_field(void* ctx, int field, const double* host, size_t n) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c || !host) return TV_ERR_ARG;
  hipSetDevice(c->device);
  // local only: no communication here (a host edit on some ranks must not make
  // only those ranks enter an exchange); the ghost planes of T / T_prev are
  // refreshed collectively at the start of every tv_step / tv_solve_T
  int rc = transfer(c, field, const_cast<double*>(host), n, 0);
  if (rc == TV_OK && hipStreamSynchronize(c->stream) != hipSuccess) rc = c->fail(TV_ERR_HIP, "sync");
  return rc;
}

int tv_get_field(void* ctx, int field, double* host, size_t n) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c || !host) return TV_ERR_ARG;
  hipSetDevice(c->device);
  return transfer(c, field, host, n, 1);
}

int tv_field_device_ptr(void* ctx, int field, void** dev_ptr, int64_t* comp_stride) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c || field < 0 || field >= TV_NUM_FIELDS) return TV_ERR_ARG;
  if (!c->f[field].ptr) return c->fail(TV_ERR_STATE, "field not materialized");
  if (dev_ptr) *dev_ptr = c->f[field].ptr;
  if (comp_stride) *comp_stride = c->f[field].space == 0 ? c->nT : c->nS;
  return TV_OK;
}

int tv_set_initial_condition(void* ctx, double T0) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c) return TV_ERR_ARG;
  hipSetDevice(c->device);
  // __set_IC_T, __set_IC_Tf, __set_IC_Tf_partial (ThermoViscoProblem.py:193-233)
  launch_fill(c->f[TV_F_T].ptr, c->nT, T0, c->stream);
  launch_fill(c->f[TV_F_T_PREV].ptr, c->nT, T0, c->stream);
  launch_fill(c->f[TV_F_TF].ptr, c->nT, T0, c->stream);
  launch_fill(c->f[TV_F_TF_PARTIAL].ptr, c->nT * 6, T0, c->stream);
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(c->stream));
  return TV_OK;
}

// ---- time-series output (ThermoViscoProblem.py:246-276, 357-364, 614-620) ----
int tv_output_open(void* ctx, const char* dir, const int* field_ids, int n_fields) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c || !dir || !field_ids || n_fields < 1) return TV_ERR_ARG;
  if (c->out) return c->fail(TV_ERR_STATE, "output already open");
  hipSetDevice(c->device);
  // mesh of the owned nodes (storage order; a partition keeps its owned planes)
  std::vector<std::vector<double>> Xs(3);
  int phys[3];
  std::vector<double> tmp;
  for (int sx = 0; sx < 3 && !c->um; ++sx) {
    Xs[sx] = storage_coords(c, sx, tmp);
    phys[sx] = c->perm[sx];
  }
  if (c->fam_T == TV_CG && c->n_parts > 1 && !c->um)
    Xs[2] = std::vector<double>(Xs[2].begin() + c->plane_begin, Xs[2].begin() + c->plane_end);
  std::string err;
  Output* o = c->um ? output_create_unstructured(dir, c->dim, c->um_xyz, c->um_cells, err)
                    : output_create(dir, c->dim, Xs, phys, err);
  if (!o) return c->fail(TV_ERR_STATE, "output: " + err);
  static const char* names[TV_NUM_FIELDS] = {
      "T", "T_prev", "T_next", "Tf", "Tf_prev", "Tf_partial", "Tf_partial_prev", "phi", "phi_next", "xi",
      "thermal_strain", "total_strain", "deviatoric_strain", "ds_partial", "dsigma_partial", "s_tilde_partial",
      "s_tilde_partial_next", "sigma_tilde_partial", "sigma_tilde_partial_next", "s_partial", "s_partial_next",
      "sigma_partial", "sigma_partial_next", "sigma", "residual", "dx"};
  for (int k = 0; k < n_fields; ++k) {
    const int id = field_ids[k];
    if (id < 0 || id >= TV_NUM_FIELDS || !c->f[id].ptr) {
      output_destroy(o);
      return c->fail(TV_ERR_ARG, "output: field not available");
    }
    const FieldInfo& fi = c->f[id];
    const bool dg = (fi.space == 0 ? c->fam_T : c->fam_S) == TV_DG;
    const int64_t n = (fi.space == 0) ? c->ownT_n : c->ownS_n;
    if (!output_add_field(o, names[id], fi.bs, dg, (size_t)n * fi.bs, err)) {
      output_destroy(o);
      return c->fail(TV_ERR_STATE, "output: " + err);
    }
  }
  if (!output_start(o, c->device, err)) {
    output_destroy(o);
    return c->fail(TV_ERR_HIP, err);
  }
  c->out = o;
  c->out_fields.assign(field_ids, field_ids + n_fields);
  return TV_OK;
}

// gathers the fields in the reference's interleaved layout into a device
// staging set on the compute stream and returns; copy and file writes overlap
// the following steps (tv_output.cpp)
int tv_output_write(void* ctx, double t) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c) return TV_ERR_ARG;
  if (!c->out) return c->fail(TV_ERR_STATE, "output not open");
  hipSetDevice(c->device);
  int set = 0;
  double* d = output_acquire(c->out, &set);
  for (size_t k = 0; k < c->out_fields.size(); ++k) {
    const FieldInfo& fi = c->f[c->out_fields[k]];
    const int64_t ndof = (fi.space == 0) ? c->ownT_n : c->ownS_n;
    const int64_t off = (fi.space == 0) ? c->ownT_off : c->ownS_off;
    const int64_t stride = (fi.space == 0) ? c->nT : c->nS;
    const bool dgsp = (fi.space == 0 ? c->fam_T : c->fam_S) == TV_DG;
    const int nl = dgsp ? (1 << c->dim) : 0;
    const int64_t ncell = dgsp ? ndof / nl : 0;
    const int64_t need = ndof * fi.bs;
    const int blocks = (int)std::min<int64_t>(std::max<int64_t>(1, (need + 255) / 256), 16384);
    hipLaunchKernelGGL(k_interleave, dim3(blocks), dim3(256), 0, c->stream, 1, d + output_offset(c->out, k), fi.ptr,
                       ndof, fi.bs, stride, off, nl, ncell);
  }
  HIPC(hipGetLastError());
  std::string err;
  if (!output_submit(c->out, set, t, c->stream, err)) return c->fail(TV_ERR_STATE, "output: " + err);
  return TV_OK;
}

int tv_output_close(void* ctx) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c) return TV_ERR_ARG;
  if (!c->out) return TV_OK;
  hipSetDevice(c->device);
  const std::string e = output_destroy(c->out);
  c->out = nullptr;
  c->out_fields.clear();
  if (!e.empty()) return c->fail(TV_ERR_STATE, "output: " + e);
  return TV_OK;
}

int tv_set_dirichlet(void* ctx, int enable, double value) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c) return TV_ERR_ARG;
  if (c->O.model_mode != TV_MODEL_PAPER)
    return c->fail(TV_ERR_STATE, "Dirichlet condition: only with model_mode = TV_MODEL_PAPER (the reference's "
                                 "own path cannot run, ThermoViscoProblem.py:236-243)");
  hipSetDevice(c->device);
  c->dir_on = enable != 0;
  c->dir_value = value;
  if (c->dir_on && c->fam_T == TV_CG && !c->dB) {
    const size_t nb = sizeof(double) * (size_t)std::max<int64_t>(1, c->nT);
    HIPC(hipMalloc(&c->dB, nb));
    HIPC(hipMalloc(&c->dtmp, nb));
    HIPC(hipMemsetAsync(c->dtmp, 0, nb, c->stream));
    HIPC(hipStreamSynchronize(c->stream));
  }
  return TV_OK;
}

int tv_sync(void* ctx) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c) return TV_ERR_ARG;
  HIPC(hipStreamSynchronize(c->stream));
  return TV_OK;
}

int tv_residual(void* ctx, const double* T_dev, double* F_dev) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c || !T_dev || !F_dev) return TV_ERR_ARG;
  hipSetDevice(c->device);
  HIPC(hipDeviceSynchronize());  // inputs written on other streams (header)
  op_residual(c, T_dev, c->f[TV_F_T_PREV].ptr, F_dev);
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(c->stream));
  return TV_OK;
}

int tv_jacobian_apply(void* ctx, const double* x_dev, double* y_dev) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c || !x_dev || !y_dev) return TV_ERR_ARG;
  hipSetDevice(c->device);
  HIPC(hipDeviceSynchronize());  // inputs written on other streams (header)
  op_japply(c, c->f[TV_F_T].ptr, x_dev, y_dev, nullptr, nullptr);
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(c->stream));
  return TV_OK;
}

int tv_jacobian_diag(void* ctx, double* d_dev) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c || !d_dev) return TV_ERR_ARG;
  hipSetDevice(c->device);
  HIPC(hipDeviceSynchronize());  // inputs written on other streams (header)
  op_diag(c, c->f[TV_F_T].ptr, d_dev, 0);
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(c->stream));
  return TV_OK;
}

int tv_precond_apply(void* ctx, const double* r_dev, double* z_dev) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c || !r_dev || !z_dev) return TV_ERR_ARG;
  if (c->n_parts > 1) return c->fail(TV_ERR_ARG, "tv_precond_apply: one partition only");
  hipSetDevice(c->device);
  HIPC(hipDeviceSynchronize());  // inputs written on other streams (header)
  const double* T = c->f[TV_F_T].ptr;
  const int64_t n = c->nT;
  hipStream_t s = c->stream;
  // the PC setup of the Newton iteration at this T
  if (!c->dggface) {
    if (!c->um && c->fam_T == TV_CG) {
      launch_cg_diag(c->cg, T, c->dinv, 1, s, c->dinv_interior);
      c->dinv_interior = true;
    } else {
      op_diag(c, T, c->dinv, 1);
    }
  }
  if (!c->mg_on) {
    launch_mg_jacobi(n, nullptr, r_dev, nullptr, nullptr, c->dinv, 1.0, z_dev, 0, s);  // z = dinv .* r
  } else {
    PcgState h{};  // running state: the V-cycle's kernels skip work once a solve is done
    HIPC(hipMemcpyAsync(c->st, &h, sizeof(PcgState), hipMemcpyHostToDevice, s));
    mg_prepare(c, T);
    HIPC(hipMemcpyAsync(c->r, r_dev, sizeof(double) * (size_t)n, hipMemcpyDeviceToDevice, s));
    if (c->dggface)  // x0 = omega0 B^-1 r (cell blocks)
      launch_dg_bsmooth(c->dg, c->st, c->r, nullptr, c->dggface, c->mg_omega0, c->mgx, 0, s);
    else
      launch_mg_jacobi(n, c->st, c->r, nullptr, nullptr, c->dinv, c->mg_omega0, c->mgx, 0, s);
    mg_apply0(c, T, nullptr);
    HIPC(hipMemcpyAsync(z_dev, c->z, sizeof(double) * (size_t)n, hipMemcpyDeviceToDevice, s));
  }
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(s));
  return TV_OK;
}

int tv_solve_T(void* ctx, int* newton_its, int* krylov_its, int* converged) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c) return TV_ERR_ARG;
  hipSetDevice(c->device);
  return newton(c, newton_its, krylov_its, converged);
}

int tv_visco_update(void* ctx) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c) return TV_ERR_ARG;
  hipSetDevice(c->device);
  if (int e = visco(c, false)) return e;
  HIPC(hipStreamSynchronize(c->stream));
  return TV_OK;
}

int tv_step(void* ctx, int thermal_only, int* newton_its, int* krylov_its) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c) return TV_ERR_ARG;
  hipSetDevice(c->device);
  int conv = 0;
  if (int e = newton(c, newton_its, krylov_its, &conv)) return e;
  if (!thermal_only) {
    if (c->ktime) HIPC(hipEventRecord(c->vev[0], c->stream));
    if (int e = visco(c, true)) return e;  // includes T_prev <- T (ThermoViscoProblem.py:378-379)
    if (c->ktime) {
      HIPC(hipEventRecord(c->vev[1], c->stream));
      HIPC(hipEventSynchronize(c->vev[1]));
      float a = 0.f;
      HIPC(hipEventElapsedTime(&a, c->vev[0], c->vev[1]));
      c->ksum[2] += a;
      c->kcnt[2] += 1;
    }
  } else {
    launch_copy(c->f[TV_F_T_PREV].ptr, c->f[TV_F_T].ptr, c->nT, c->stream);
  }
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(c->stream));
  return TV_OK;
}

int tv_comm_unique_id_size(void) { return (int)sizeof(ncclUniqueId); }

int tv_comm_get_unique_id(char* id_out) {
  if (!id_out) return TV_ERR_ARG;
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) {
    set_global_error(std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
    return TV_ERR_COMM;
  }
  std::memcpy(id_out, &id, sizeof(id));
  return TV_OK;
}

int tv_comm_init(void* ctx, const char* id, int n_ranks, int rank) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c || !id) return TV_ERR_ARG;
  if (n_ranks != c->n_parts || rank != c->part)
    return c->fail(TV_ERR_ARG, "communicator size/rank must match the mesh partition (n_parts/part)");
  hipSetDevice(c->device);
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  NCCLC(ncclCommInitRank(&c->comm, n_ranks, uid, rank));
  c->nranks = n_ranks;
  c->rank = rank;
  // bring ghost planes of the state up to date
  if (int e = halo(c, c->f[TV_F_T].ptr)) return e;
  if (int e = halo(c, c->f[TV_F_T_PREV].ptr)) return e;
  HIPC(hipStreamSynchronize(c->stream));
  return TV_OK;
}

int tv_comm_init_host(void* ctx, int n_ranks, int rank, tv_host_allreduce_fn allreduce_fn,
                      tv_host_sendrecv_fn sendrecv_fn, void* user) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c || !allreduce_fn || !sendrecv_fn) return TV_ERR_ARG;
  if (n_ranks != c->n_parts || rank != c->part)
    return c->fail(TV_ERR_ARG, "communicator size/rank must match the mesh partition (n_parts/part)");
  hipSetDevice(c->device);
  c->nranks = n_ranks;
  c->rank = rank;
  c->host_allreduce = allreduce_fn;
  c->host_sendrecv = sendrecv_fn;
  c->host_user = user;
  if (c->fam_T == TV_CG) {
    const int64_t plane = (int64_t)c->cg.n0 * c->cg.n1;
    HIPC(hipHostMalloc(&c->h_halo, sizeof(double) * 4 * (size_t)plane));
  }
  if (int e = halo(c, c->f[TV_F_T].ptr)) return e;
  if (int e = halo(c, c->f[TV_F_T_PREV].ptr)) return e;
  HIPC(hipStreamSynchronize(c->stream));
  return TV_OK;
}

int tv_halo_exchange(void* ctx, int field) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c || field < 0 || field >= TV_NUM_FIELDS || !c->f[field].ptr) return TV_ERR_ARG;
  if (c->f[field].space != 0 || c->f[field].bs != 1) return c->fail(TV_ERR_ARG, "halo exchange: scalar T-space fields only");
  if (int e = halo(c, c->f[field].ptr)) return e;
  HIPC(hipStreamSynchronize(c->stream));
  return TV_OK;
}

int tv_kernel_bytes(void* ctx, int kernel, double* bytes) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c || !bytes) return TV_ERR_ARG;
  const double n = (double)c->ownT_n;
  const int dd = c->dim * c->dim;
  switch (kernel) {
    case 0:  // J(T) x : read x, write y (geometry implicit, T only on boundary nodes)
    case 10:  // the same, timed with the Infinity Cache flushed (tv_time_kernel)
      // unstructured: + the assembled cell operator (8 B value + 4 B column per
      // stored SELL entry, padding included) and the Robin data of the boundary
      *bytes = c->um ? 16.0 * n + 12.0 * (double)um_nnz(c->umd) : 16.0 * n;
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
      // level 0: J x0 (16), restriction reads r, w (16), prolongation x0 -> x (16),
      // then CG: J x with the post-smoothing in its epilogue (x, r, dinv in, z out: 32),
      // DG: J x (16) + the cell-block post-smoothing (x0, r, w in, z out: 32)
      double b = (c->mg_dg ? 16.0 + 16 + 16 + 16 + 32 : 16.0 + 16 + 16 + 32) * n;
      for (size_t l = 0; l < c->mg.size(); ++l) {
        const double nl = (double)c->mg[l].n;
        b += 24.0 * nl;  // the restriction's outputs b, x (pre-smoothing) and the dinv it reads
        if (l + 1 < c->mg.size())  // J x (16), restriction reads (16), partial J x (16), prolongation in (16),
          b += (16.0 + 16 + 16 + 16 + 24) * nl;  // post-smoothing operands b, w, dinv (24)
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
  if (kernel == 11) {  // V-cycles on the current state (solver state reset: not converged)
    if (!c->mg_on) return c->fail(TV_ERR_ARG, "kernel 11: preconditioner GMG not enabled");
    PcgState h{};
    h.max_it = 1 << 30;
    HIPC(hipMemcpyAsync(c->st, &h, sizeof(PcgState), hipMemcpyHostToDevice, c->stream));
    mg_prepare(c, c->f[TV_F_T].ptr);
  }
  auto one = [&]() -> int {
    int np = 0;
    switch (kernel) {
      case 11: mg_apply0(c, c->f[TV_F_T].ptr, nullptr); return TV_OK;
      case 0: op_japply(c, c->f[TV_F_T].ptr, c->pA, c->w, nullptr, nullptr); return TV_OK;
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
  if (kernel == 10) {
    // J x with the Infinity Cache flushed before every launch: a 512 MiB write
    // (2x the 256 MiB L3) then a read sweep of the same buffer, so the cache
    // holds clean lines (no write-backs of the flush competing with the timed
    // launch), HIP events around each launch alone (SURVEY.md section 8(d) H7:
    // the HBM figure, not the cache-assisted one)
    const size_t fl = (size_t)512 << 20;
    void* flush = nullptr;
    HIPC(hipMalloc(&flush, fl));
    std::vector<hipEvent_t> ev(2 * (size_t)reps);
    for (auto& e : ev) HIPC(hipEventCreate(&e));
    op_japply(c, c->f[TV_F_T].ptr, c->pA, c->w, nullptr, nullptr);  // warm-up
    for (int i = 0; i < reps; ++i) {
      HIPC(hipMemsetAsync(flush, i & 0xff, fl, c->stream));
      hipLaunchKernelGGL(k_read_sweep, dim3(1024), dim3(kBlock), 0, c->stream, static_cast<const double*>(flush),
                         (int64_t)(fl / sizeof(double)), c->partials);
      HIPC(hipEventRecord(ev[2 * i], c->stream));
      op_japply(c, c->f[TV_F_T].ptr, c->pA, c->w, nullptr, nullptr);
      HIPC(hipEventRecord(ev[2 * i + 1], c->stream));
    }
    HIPC(hipEventSynchronize(ev.back()));
    double sum = 0.0;
    for (int i = 0; i < reps; ++i) {
      float t = 0.f;
      HIPC(hipEventElapsedTime(&t, ev[2 * i], ev[2 * i + 1]));
      sum += t;
    }
    for (auto& e : ev) hipEventDestroy(e);
    HIPC(hipFree(flush));
    *ms = sum / reps;
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
  *ms_avg = c->kcnt[k] ? c->ksum[k] / (double)c->kcnt[k] : 0.0;
  if (launches) *launches = c->kcnt[k];
  return TV_OK;
}

int tv_pcg_variant(void* ctx, int* variant) {
  Ctx* c = static_cast<Ctx*>(ctx);
  if (!c || !variant) return TV_ERR_ARG;
  *variant = c->cgs ? TV_PCG_SINGLE_REDUCTION : TV_PCG_KSPCG;
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

}  // extern "C"
