// Host runtime of libtvfem.so: the per-context state (struct Ctx) shared by
// the runtime's translation units, and the functions they call across files.
// Not part of the C-ABI (include/tvfem.h).
//
//   tv_context.cpp  context creation / destruction, mesh partition, device
//                   state, field transfer, output and Dirichlet settings
//   tv_comm.cpp     halo exchanges and reductions (RCCL or host-staged)
//   tv_solver.cpp   Newton + Krylov drivers (KSPCG, single-reduction), the
//                   Dirichlet lifting, the viscoelastic step, the operators
//   tv_mgsolve.cpp  geometric-multigrid hierarchy and the preconditioned solve
//   tv_measure.cpp  in-solve kernel timing, algorithmic bytes, timed launches
//
// Reference mapping (file:line under /root/reference):
//   Ctx construction      ThermoViscoProblem.__init__ (ThermoViscoProblem.py:24-58)
//   initial condition     _set_initial_condition (:187-233)
//   tv_solve_T            _solve_T (:384-391) -> dolfinx NewtonSolver [3P]
//                         configured at _setup_solver (:330-346)
//   tv_visco_update       _solve_Tf .. _solve_stress (:393-595)
//   tv_step               solve_timestep (:367-381) without _write_output
#pragma once
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

struct FieldInfo {
  double* ptr = nullptr;
  void* base = nullptr;  // the allocation (ptr = base + the field's stagger)
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
  // partitioned contexts (tv_mgdist.cpp): a distributed level is this rank's
  // slab of the global level with one ghost plane per interface (dist); a
  // replicated level is the whole global level on every rank.  first2 = global
  // plane of local plane 0 along storage axis 2; [inj0, inj1) = the local
  // planes whose T this rank injects (its coarse planes)
  bool dist = false;
  int first2 = 0;
  int inj0 = 0, inj1 = 0;
  double* mask = nullptr;    // the level above the replicated ones: 1 owned / 0 ghost
  // the fused residual restriction INTO this level (RRArgs, tv_mg.hip): rr.on
  // where the transfer's geometry allows it (one partition, tv_mgsolve.cpp)
  RRArgs rr{};
};

// level l >= 1 of the algebraic multigrid (tv_amg.cpp): A_l, the prolongation
// into level l - 1 (rows of that level) and R = P^T; the stored SELL entries
struct AmgLevel {
  int64_t n = 0;
  Sell A, P, R;
  UmGrid sg{};  // geometric levels: A as a half stencil (sg.J14 != nullptr: applied so instead of A)
  // the first geometric level: its grid and the fine one's (the level-0
  // transfers applied by index arithmetic, launch_geo_*); geo0 = false: SELL P, R
  bool geo0 = false;
  int64_t gfine[3] = {0, 0, 0}, gcoarse[3] = {0, 0, 0};
  int64_t a_nnz = 0, p_nnz = 0, r_nnz = 0;
  double omega = 0.0;
  double *dinv = nullptr, *b = nullptr, *x = nullptr, *w = nullptr;
};

struct Ctx {
  std::string err;
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  hipEvent_t evp[2] = {nullptr, nullptr};  // PCG convergence polls (double-buffered)
  hipEvent_t evn[2] = {nullptr, nullptr};  // Newton: ||dx|| and the decision copied to the host (slot)
  const double* nrm_dev = nullptr;          // ... from here (||dx||^2, final on every rank behind evn)
  // the device's Newton test (queue_newton_norm), two slots by the parity of
  // the Newton iteration: ngate[2 s] = ||dx||^2, ngate[2 s + 1] = the decision;
  // ngate[4] = ||dx_1||^2 (r0 of the incremental test, recorded on the device).
  // gate_dev points at the decision of the last queued norm (nullptr:
  // iteration 1, no test); solve_gate is the decision the next solve's state
  // launch is gated on (a solve queued before the host read that decision)
  double* ngate = nullptr;
  const double* gate_dev = nullptr;
  const double* solve_gate = nullptr;
  int newton_slot = 0;
  bool newton_first = true;
  // queue the predicted next Newton iteration's solve ahead of the host's read
  // (multigrid paths); TVFEM_NEWTON_AHEAD=0 at creation: wait at every boundary
  // (a test / measurement switch, tests/test_multigrid.py)
  bool newton_ahead = true;
  tv_params P{};
  tv_options O{};
  int dim = 1;
  int fam_T = TV_CG, fam_S = TV_CG;
  int perm[3] = {0, -1, -1};  // storage axis -> physical axis (-1 degenerate)
  int n_parts = 1, part = 0;
  // global / local sizes
  int Nnode_glob[3] = {1, 1, 1};  // per storage axis
  int Ncell_glob[3] = {0, 0, 0};
  int ghost_depth = 1;  // ghost planes per interface of the fine CG slab (3: deep ghosts, tv_mgdist.cpp)
  int plane_begin = 0, plane_end = 0;  // owned global planes (CG) / cell layers (DG) along storage axis 2
  CgGrid cg{};
  bool dinv_interior = false;  // dinv holds the T-independent interior diagonal (CG march path)
  DgGrid dg{};
  int64_t nT = 0, nS = 0;          // local dofs incl. ghosts
  int64_t ownT_off = 0, ownT_n = 0;
  int64_t ownS_off = 0, ownS_n = 0;
  int64_t globT_off = 0, globS_off = 0;
  // mixed families on a slab partition (setup_mixed_part): 1 = DG T / CG sigma
  // (main.py), 2 = CG T / DG sigma; outT_n / outS_n: dofs each space writes to
  // the part's output mesh (the nodes of its owned cell layers)
  int mixed_part = 0;
  int64_t outT_n = 0, outS_n = 0;
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
  // the single-reduction (Chronopoulos-Gear) form of the distributed GMG-PCG
  // on a deep-ghost slab (tv_mgdist.cpp): s = A p by recurrence
  bool mg_cgs = false;
  double* mg_s = nullptr;
  double* dggface = nullptr; // DG level 0: facet means of dg(T) for the cell-block Jacobi smoother
  // partitioned GMG (tv_mgdist.cpp): levels 0 .. mg_A - 1 are distributed over
  // the partitions, mg_A .. the coarsest are replicated on every rank
  int mg_A = 0;
  // options.mg_coupling LOCAL (block Jacobi): every level is this partition's
  // own slab, the transfers stop at its owned planes, no exchange in the V-cycle
  bool mg_local = false;
  double* mg_mask0 = nullptr;  // level 0 restriction mask when mg_A == 1 (1 owned / 0 ghost)
  double* h_big = nullptr;     // pinned staging of vector all-reduces (host-staged transport)
  size_t h_big_n = 0;
  // unstructured mesh (tv_create_unstructured, tv_um.hip)
  bool um = false;
  UmGrid umg{};
  std::vector<double> um_xyz;        // host copy: 3 per vertex
  std::vector<int64_t> um_cells;     // host copy: 2^dim per cell (input order)
  UmDevice* umd = nullptr;            // assembled operators, facet data (tv_um.hip)
  unsigned char* um_bmask = nullptr;  // boundary vertices (Dirichlet mode)
  // algebraic multigrid (options.preconditioner = TV_PC_AMG, unstructured, tv_amg.cpp)
  bool amg_on = false;
  std::vector<AmgLevel> amg;
  std::vector<void*> amg_bufs;
  // partitioned unstructured mesh (tv_create_unstructured_part): owned vertices
  // first, ghosts grouped by owner; per neighbour k: the ghosts received from
  // um_peer[k] at [nown + um_roff[k], + um_rcnt[k]), the owned values sent to it
  // packed at [um_soff[k], + um_scnt[k]) of um_sbuf (indices um_sidx)
  int64_t um_own_cells = 0;
  std::vector<int> um_peer;
  std::vector<int64_t> um_rcnt, um_roff, um_scnt, um_soff;
  int64_t* um_sidx = nullptr;
  double* um_sbuf = nullptr;
  std::vector<int> out_fields;
  double *cr[2] = {nullptr, nullptr}, *cs[2] = {nullptr, nullptr}, *cw1 = nullptr;
  double* wsend = nullptr;
  double* dg_sbuf = nullptr;  // partitioned DG: the first and the last owned cell layer, packed for the halo
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
  bool comm_stub = false;    // tv_comm_init_stub: measurement of one rank's share, no transport
  // tv_comm_init_loopback: a ONE-rank RCCL communicator; every neighbour of the
  // partition is this rank itself (peer 0), so the production RCCL groups run
  // with self send/recv pairs and one-rank all-reduces (transport test)
  bool comm_self = false;
  // partitioned unstructured mesh: T-space / sigma-space fields written from
  // the host since the last step (tv_set_field writes owned dofs only); their
  // ghosts are refreshed collectively at the next step (refresh_dirty_ghosts)
  uint32_t ghost_dirty = 0;
  double* d_dirty = nullptr;
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
  bool vev_pending = false;          // the last step's visco events not yet read
  double ksum[3] = {0.0, 0.0, 0.0};  // ms: fused matvec, PCG update, visco update
  int64_t kcnt[3] = {0, 0, 0};
  // stats
  int last_newton = 0, last_krylov = 0;
  double last_dx = 0.0;
  int last_conv = 0;  // the last Newton solve met its test (tv_last_converged)
  int pcg_hint = 0;
  // multigrid solves: the Krylov count of the Newton iteration with the same
  // index in the previous time step (the solves of a step take a repeating
  // pattern of counts, e.g. 6 5 5 4: the previous solve's count over-queues
  // early-exit iterations, ~25 launches each), and the index of the current one
  int mg_hint[16] = {0};
  int jac_hint[16] = {0};  // the same for the Jacobi-PCG solves
  int newton_k = 0;
  int newton_pred = 0;  // the previous step's Newton count (speculative residual, newton())

  int fail(int code, const std::string& m) {
    err = m;
    return code;
  }
};

// component stride of the fields of a space: the dof count rounded up to 64
// values (512 B), so that every component of a blocked field starts aligned
// (C4's 8,200,851 nodes put components 1.. at 152-byte offsets: each wave's
// 512-byte access then touched five 128-byte lines instead of four)
inline int64_t field_stride(const Ctx* c, int space) {
  const int64_t n = space == 0 ? c->nT : c->nS;
  return (n + 63) / 64 * 64;
}

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

constexpr int64_t kCgsAutoMaxNodes = 3000000;  // AUTO Krylov form: single reduction up to this slab size
constexpr int64_t kCgsAutoMaxNodes1 = 1500000;  // ... and on one partition up to this size (Jacobi)
constexpr int kTsCap = 1 << 15;                // timestamp slots of the in-solve kernel timing

// ---- tv_amg.cpp ----
int amg_setup(Ctx* c);
int amg_setup_part(Ctx* c);  // collective (partitioned unstructured mesh), at the first solve
int amg_apply0(Ctx* c, const RedTail* tail);
double amg_cycle_bytes(const Ctx* c);

// ---- tv_context.cpp ----
void set_global_error(const std::string& m);
void axis_coefs(const std::vector<double>& X, int first, int count, std::vector<double>& out);
const std::vector<double>& storage_coords(Ctx* c, int s, std::vector<double>& tmp);
bool storage_perm(const tv_mesh_desc* m, int perm[3]);
void part_planes(int N2, int P, int p, int* b0, int* b1);  // owned planes [b0, b1) of partition p of P
int build_cg_grid(Ctx* c, int d, const std::vector<double> (&X)[3], int first2, int n2, int g_lo, int g_hi,
                  bool bnd2lo, bool bnd2hi, CgGrid& g, double** coef, int64_t** bnodes, double** ffbuf);
int transfer(Ctx* c, int field, double* host, size_t n, int dir);

// ---- tv_comm.cpp ----
bool multi_rank(const Ctx* c);
int halo(Ctx* c, double* v);  // ghost planes of a T-space vector of the fine grid
int halo_grid(Ctx* c, const CgGrid& g, double* v);  // ghost planes of a vector of grid g (a GMG level)
int allreduce_vec(Ctx* c, double* v, int64_t n);
int halo_um(Ctx* c, double* v);  // ghosts of a partitioned unstructured mesh's T-space vector
int comm_check(Ctx* c, int64_t* n_checked, int64_t* n_bad);  // tv_comm_check
int allreduce_halo(Ctx* c, double* sums, int n, double* v);
int visco_timing_flush(Ctx* c);  // tv_solver.cpp  // one RCCL group: n-scalar sum + halo(v)  // sum over the ranks of a device vector, in place
int allreduce(Ctx* c, double* v, int n);
int reduce_logic(Ctx* c, int n, int W, int kind, int check_done);  // records -> (all-reduce) -> scalar logic
int cgs_raxis(const Ctx* c);
int cgs_exchange(Ctx* c, double* wout, const double* fout);
// a partitioned context must have its transport before it solves (the solve
// would otherwise run on stale ghosts with local-only norms)
int require_comm(Ctx* c, const char* what);
// partitioned unstructured mesh: the ghost values of every field some rank
// wrote from the host since the last step, from their owners (collective)
int refresh_dirty_ghosts(Ctx* c);

// ---- tv_solver.cpp ----
void op_residual(Ctx* c, const double* T, const double* Tp, double* F);
void op_diag(Ctx* c, const double* T, double* d, int invert);
void op_japply(Ctx* c, const double* T, const double* x, double* y, double* partials, int* np);
bool op_japply_fused(Ctx* c, const double* T, int* np, const RedTail* tail = nullptr, int it = 0);
PcgState pcg_state_init(const Ctx* c);
int ts_flush(Ctx* c);
CgsBuffers cgs_buffers(Ctx* c, const double* T, int it);
// step_end (tv_step): 0 none, 1 the visco update, 2 T_prev <- T (thermal only).
// At the Newton iteration the last step predicts to be the final one, the step's
// end is queued before the host reads ||dx||, gated on the device's Newton test
// (NewtonGate); *end_queued tells tv_step that it ran (the step is done).  On
// the multigrid paths an iteration the last step predicts is queued before the
// host reads the previous test, its solve gated on that test (solve_gate)
int newton(Ctx* c, int* out_its, int* out_kits, int* out_conv, int step_end = 0, bool* end_queued = nullptr);
int visco(Ctx* c, bool copy_Tprev, const NewtonGate& gate = NewtonGate{});
// the Newton iteration's ||dx||^2 (final on every rank at nrm2) and the device's
// convergence decision (k_newton_test) to the host slot newton_slot; records evn[slot]
int queue_newton_norm(Ctx* c, const double* nrm2);
// dev_src -> pinned host_dst on the context stream (a one-wave kernel; bytes % 4 == 0)
int publish(Ctx* c, void* host_dst, const void* dev_src, size_t bytes);
void launch_bc_mask(Ctx* c, double* dinv);  // dinv = 0 on the Dirichlet-constrained rows

// ---- tv_mgsolve.cpp ----
int mg_setup(Ctx* c);
int mg_prepare(Ctx* c, const double* T);
int mg_dg_weight(Ctx* c, const double* T);
int mg_apply0(Ctx* c, const double* T, const RedTail* tail);
// post: queue the Newton iteration's post-solve group (launch_post_group, ||dx||
// copied to h_sums, evn[slot] recorded) behind every batch, gated on the device state
int pcg_solve_mg(Ctx* c, const double* T, int* its, int* reason, bool post = false);
bool mg_next_level(const std::vector<double> (&Xp)[3], double da, bool automatic, std::vector<double> (&Xc)[3],
                   std::vector<char> (&is_c)[3], int coarse[3]);
void mg_axis_tables(const std::vector<double>& Xf, const std::vector<char>& is_c, std::vector<int>& pi,
                    std::vector<double>& pw, std::vector<int>& ri, std::vector<double>& rw);
int mg_level_vectors(Ctx* c, MgLevel& L);
double mg_gershgorin(const std::vector<double> (&X)[3], double dt_alpha);
double mg_omega(double b);
void mg_level(Ctx* c, size_t l);
template <class T>
int mg_upload(Ctx* c, MgLevel& L, const std::vector<T>& h, const T** out) {
  void* p = nullptr;
  HIPC(hipMalloc(&p, sizeof(T) * std::max<size_t>(1, h.size())));
  L.bufs.push_back(p);
  HIPC(hipMemcpy(p, h.data(), sizeof(T) * h.size(), hipMemcpyHostToDevice));
  *out = static_cast<const T*>(p);
  return TV_OK;
}

// ---- tv_mgdist.cpp (GMG on a slab-partitioned box) ----
int mg_setup_dist(Ctx* c);
int pcg_solve_mg_dist(Ctx* c, const double* T, int* its, int* reason, bool post = false);
int mg_prepare_dist(Ctx* c, const double* T);
void fine_window(const Ctx* c, int64_t* off, int64_t* n);
int mg_apply0_dist(Ctx* c, const double* T, const RedTail* tail);

}  // namespace tv
