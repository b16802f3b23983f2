// Internal definitions shared by the HIP kernels and the host runtime of
// libtvfem.so.  Not part of the C-ABI (see include/tvfem.h).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <string>
#include <vector>

#include "tvfem.h"

namespace tv {

constexpr int kWave = 64;         // CDNA wavefront
constexpr int kSeg = kWave - 2;   // outputs per wave of the x-row stencil kernels
constexpr int kBlock = 256;       // 4 waves

// Per-node coefficients of one storage axis of a rectilinear grid: the
// assembled 1D P1 mass (lo, diag, up), 1D stiffness (lo, diag, up), and the
// lengths of the cells below / above the node (0 where no cell exists).
// A degenerate axis (1 node) carries M = (0, 1, 0), K = 0, h = 0.
enum { C_MLO = 0, C_MDI, C_MUP, C_KLO, C_KDI, C_KUP, C_HLO, C_HHI, C_NCOEF };

// Grid of the CG1 (Q1 / P1) temperature space on one partition.  Storage axis
// 0 is physical x (fastest), storage axis 2 is the partition axis (slowest);
// local node index = i + n0*(j + n1*k).  Along axis 2 the local array holds the
// owned planes plus g_lo / g_hi ghost planes towards the neighbouring
// partitions: one, or three on the fine grid of a distributed multigrid solve
// (deep ghosts, tv_mgdist.cpp), whose kernels then write every plane of the
// write window [w_begin, w_end) -- all local planes but the outermost ghost
// plane on each side -- and reduce over the owned planes only.
// Operands of the multigrid post-smoothing fused into the Jacobian march
// (k_cg_march POST): z = x + omega dinv (r - J x)
struct PostArgs {
  const double* r;
  const double* dinv;
  double omega;
};

constexpr int kDeepGhosts = 3;  // ghost planes of a deep-ghost fine slab

struct CgGrid {
  int n0, n1, n2;             // local node counts per storage axis (n2 incl. ghosts)
  int k_begin, k_end;         // owned planes along axis 2, local indexing
  int g_lo, g_hi;             // ghost planes present below / above
  int w_begin, w_end;         // write window (= [k_begin, k_end) with one ghost plane)
  int deg1, deg2;             // storage axis 1 / 2 degenerate (single node)
  int bnd[3][2];              // face of storage axis a at side s is a physical boundary here
  const double* coef[3];      // device, C_NCOEF doubles per local node per axis
  double dt, dt_alpha, dt_f;  // dt, dt*alpha, dt*f
  double a_rad, a_conv;       // 0.001*sigma*epsilon, 0.001*htc
  double T_amb, T_amb4;
  const int64_t* bnodes;      // owned nodes on physical boundary faces (3D marching path)
  int64_t n_bnodes;
  // Robin facet Jacobian terms per physical face f = 2*axis + side (3D marching
  // path): one value per face node, fface[f][c_t1 + fn1[f] * c_t2] (tangential
  // axes t1 < t2), rewritten by k_cg_faces before every Jacobian application
  double* fface[6];
  int fn1[6], fn2[6];
  // the six face arrays are one contiguous buffer per parity (ffbuf[0] holds
  // fface[] above; ffbuf[1] is the second set of the single-reduction PCG,
  // which reads one set while it writes the other); ffoff[f] = offset of face
  // f in doubles, -1 where face f is not a physical boundary of this partition
  double* ffbuf[2];
  int64_t ffoff[6];
  int64_t ffsize;
};

// Grid of the DG1 temperature space: cells per storage axis; dof layout is
// component-major [local vertex l][local cell], l = a + 2b + 4c (storage axes).
struct DgGrid {
  int c0, c1, c2;             // local cell counts (c2 incl. ghost layers)
  int k_begin, k_end;         // owned cell layers along axis 2
  int deg1, deg2;
  int bnd[3][2];
  const double* h[3];         // device: cell length per local cell per axis
  const double* ih[3];        // device: 1 / h (the tile kernels: no FP64 divisions per cell)
  double hdiam_inv;           // unused for rectilinear non-uniform (per-cell below)
  double dt, dt_alpha, dt_f;
  double a_rad, a_conv;
  double T_amb, T_amb4;
  double penalty;             // SIPG penalty (ThermoViscoProblem.py:313)
  // 3D Jacobian kernel: 1 = marching tiles (k_dg_tile) of 8 computing waves whose
  // edge waves load the halo rows, `tile_chunk` planes per workgroup (default);
  // 0 = one thread per cell (k_dg_cells, the reference the tile kernel is
  // tested against); tv_options.dg_kernel / dg_tile_chunk
  int tile, tile_chunk;
  // partitions along storage axis 2: local layers [0, c2) = k_begin ghost
  // layers below the owned ones [k_begin, k_end) and c2 - k_end above.  The
  // owned layers' dofs come first, component-major over the `own` owned cells
  // ([l][owned cell], so the owned dofs are one contiguous range as the Krylov
  // vector kernels need); each ghost layer's follow, component-major over its
  // c0 c1 cells, from offset gofs[0] (below) / gofs[1] (above).  One partition:
  // own = c0 c1 c2 -- the plain [l][cell] layout.
  int64_t own;
  int64_t gofs[2];
};

// two-level in-kernel reduction tails (tv_device.h fused_reduce_tail): kShards
// shard counters + 1 top counter per tail; two tails per context (matvec,
// update), rounded up
constexpr int kShards = 8;
constexpr int kTailCounters = kShards + 1;
constexpr int kCounterWords = 32;
constexpr int kUpdateCounter = 2 * kTailCounters;  // the multigrid update's commit ticket (lagged logic)
static_assert(kUpdateCounter < kCounterWords, "counter words");

// Device-resident scalars of one PCG solve (PETSc KSPCG restated, preconditioned norm).
struct PcgState {
  double beta, betaold, dpi, dpiold, a, dp, rnorm0, ttol;
  double rtol, atol, dtol;
  int it, done, reason, max_it;
  int post;                   // the post-solve group queued behind the batches has run (pcg_solve_mg)
  int accept_its;             // ksp_fixed_its > 0: a solve ending at max_it (DIVERGED_ITS) is a good outcome
  int relaxed;                // the measurement stub (tv_comm_init_stub): no indefiniteness breakdowns --
                              // its zeroed ghosts make the slab's operator inconsistent, the fixed
                              // iterations are timed, not used
  double dx_norm2;            // ||dx||^2 of the last Newton update
  double a_prev;              // step length of the previous iteration (dx is updated every 2nd)
  // single-reduction form (k_cgs_march): gamma = (r, z) and eta = (p, A p) of
  // the last iteration (PETSc's beta and dpi); a, beta as above
  double gamma, eta;
};

// In-kernel reduction tail (last-arriving workgroup reduces the partial records
// of the launch (and of a preceding launch) and runs the PCG scalar logic).
struct RedTail {
  unsigned* counter;          // nullptr: no tail (separate reduce launch)
  const double* partials;
  double* out;                // reduced sums (read by RCCL allreduce on multi-GPU)
  PcgState* st;
  int kind;                   // 0 none, 1 init, 2 p.w, 3 update, 4 / 5 single-reduction init / iteration
  // in-solve kernel timing (tv_kernel_timing), or nullptr: ts[0] = REALTIME
  // clock when workgroup 0 starts, ts[1] = when the tail workgroup finishes
  uint64_t* ts;
  // lagged scalar logic (multi-rank, tv_device.h lagged_state): the launch
  // forms the state from *st and the all-reduced sums `lag` (logic lag_kind)
  // at its start and its tail commits it -- the one-thread logic launch after
  // the previous all-reduce is folded into this launch
  const double* lag = nullptr;
  int lag_kind = 0;
};

enum PcgReason {
  R_RUNNING = 0,
  R_CONV_RTOL = 2, R_CONV_ATOL = 3,
  R_DIV_ITS = -3, R_DIV_DTOL = -4, R_DIV_INDEF_PC = -8, R_DIV_NANINF = -9, R_DIV_INDEF_MAT = -10,
  // not a PETSc reason: a solve queued ahead of the Newton test of the previous
  // iteration, which found Newton converged (k_set_state's gate): nothing ran
  R_SKIPPED = -100,
};

// Viscoelastic constants (ViscoelasticModel.py:15-83), uploaded as a kernel argument.
struct ViscoConst {
  double H_over_Rg, inv_Tb, dt, half_dt, alpha_s, dalpha, inv_dim;
  double lambda_m[6], m_n[6], lambda_g[6], g_n[6], lambda_k[6], k_n[6];
  double chi;   // ViscoelasticModel.py:15 (Eq. 25, paper mode only)
  int paper;    // model_mode: 0 reference semantics (quirks Q1-Q4 kept), 1 paper
};

// Pointers of the viscoelastic state (component-major, stride = n_local).
// the incremental Newton test of newton(), decided ONCE on the device
// (k_newton_test, tv_solver.cpp): *flag != 0 when sqrt(||dx||^2) / r0 < rtol or
// sqrt(||dx||^2) < atol; the host copies the same flag and takes it as its own
// convergence decision, so a gated launch and the host never disagree
// (flag == nullptr: always open)
struct NewtonGate {
  const double* flag = nullptr;
};
#ifdef __HIPCC__
__device__ __forceinline__ bool newton_gate_open(const NewtonGate& g) {
  return g.flag == nullptr || *g.flag != 0.0;
}
#endif

struct ViscoFields {
  int64_t n;                  // dofs processed (owned range length)
  int64_t off_T, off_S;       // first processed dof in T-space / sigma-space arrays
  int64_t sT, sS;             // component strides of T-space / sigma-space fields
  const int* map;             // sigma dof -> T dof (mixed families) or nullptr
  double* T; double* Tp; double* Tn; double* phi; double* phin; double* xi;
  double* Tf; double* Tfp;    // Tf (== Tf_prev), Tf_partial (== Tf_partial_prev)
  double* th; double* tot; double* dev;          // strains (materialize=all)
  double* ds; double* dsig;                      // increments (materialize=all)
  double* st; double* sgt;                       // s_tilde, sigma_tilde (state)
  double* sp; double* sgp;                       // s, sigma partial (materialize=all)
  double* sigma;                                 // total stress (state)
  double* Tfo;                                   // paper mode, mixed families: previous Tf per T dof (work)
  int copy_Tprev;             // fuse T_prev <- T (same family, single pass)
  // device word: 0 = s_tilde and sigma_tilde hold +0.0 at every dof (quirk Q3
  // keeps them there), so the update neither reads nor rewrites them; 1 = general
  int* tflag;
  // Newton gate (queued before the host has read ||dx||, newton()): the launch
  // runs only if the Newton test on the device's ||dx||^2 passes -- the same
  // operations as the host's test, so both decide alike; nullptr: ungated
  NewtonGate gate;
};

// Unstructured CG1 mesh (quadrilaterals / hexahedra of any shape, tv_um.hip).
// The cell part of J(T) = M + dt alpha K does not depend on T: it is assembled
// once, at context creation, into SELL-64 (sliced ELLPACK, one 64-row slice
// per wavefront, column-major inside a slice so a wave's loads are coalesced).
// The T-dependent Robin terms are evaluated on the fly from per-facet
// quadrature weights, row by row (boundary rows only).
struct UmGrid {
  int dim;
  int64_t nv, nc, nf, nslice;
  int64_t nrow;          // rows computed: all nv, or a partition's owned vertices (numbered first)
  // assembled cell operators (entry k of row r: soff[r / 64] + 64 k + r % 64)
  const int64_t* soff;   // nslice + 1
  const int* cols;
  const double* V;       // M + dt alpha K  (J x)
  const double* M;       // mass            (residual)
  const double* K;       // dt alpha K      (residual)
  const double* bvec;    // int phi_i       (f term of the residual)
  const double* vdiag;   // diag V
  // topologically structured hexahedra (vertex i + s1 j + s2 k, the box's cells,
  // any coordinates -- a jittered / warped plate, an extruded or transfinite
  // gmsh mesh): the operators as stencil slots, no column indices.  Slot q =
  // (di + 1) + 3 (dj + 1) + 9 (dk + 1) couples row r to column r + o_q, o_q =
  // di + s1 dj + s2 dk; the operators are symmetric and o_{26-q} = -o_q, so only
  // the upper half q = 13 .. 26 is stored, X14[(q - 13) nv + r], and the lower
  // slot q of row r is the upper slot 26 - q of row r + o_q (read from the
  // neighbour row's stream, a cache hit): 112 B per row and operator from HBM
  // instead of ~330 B of SELL.  J14 = V14 with the Robin facet Jacobian of J(T)
  // folded into the boundary rows' slots (launch_um_robin_fold, once per Newton
  // iteration): the J x kernels then run no facet quadrature (brow: the nbr
  // boundary rows).  M14 / K14: the residual's mass and dt alpha K, the same
  // way (marched along the planes, k_um_res14).  nullptr: SELL only.
  const double* V14;
  double* J14;
  const double* M14;
  const double* K14;
  const int64_t* brow;
  int64_t nbr;
  int64_t s1, s2;
  // Robin terms
  const int* fv;         // [m][facet] facet vertex ids, facet-local tensor order
  const double* fw;      // [q][facet] w_q |J_s|(q), 3^(d-1) points
  const int* boff;       // nv + 1: boundary incidences of each row
  const int* binc;       // 4 facet + m
  double dt, dt_alpha, dt_f;
  double a_rad, a_conv;
  double T_amb, T_amb4;
};

// A sparse operator on the device: SELL-64 (entry k of row r: soff[r / 64] +
// 64 k + r % 64; padding entries: value 0, column 0) or, csr = 1, CSR (soff =
// the row pointer) -- the fine unstructured operator and the algebraic
// multigrid's coarse operators (double), prolongations (CSR) and restrictions
// (SELL), the transfers with float32 values (fp32 = 1: vals is a float array)
struct Sell {
  int64_t nrow = 0, ncol = 0, nslice = 0;
  const int64_t* soff = nullptr;
  const int* cols = nullptr;
  const void* vals = nullptr;
  const int* perm = nullptr;  // SELL: stored position -> row (nullptr: identity)
  int csr = 0, fp32 = 0;
};
int amg_num_blocks(const Sell& M);  // partial records of launch_amg_prolong0
// y = A x
void launch_amg_apply(const Sell& A, const PcgState* st, const double* x, double* y, hipStream_t s);
// b_c = R (x - x2) (x2 may be null), x_c = omega_c dinv_c b_c (x_c may be null)
void launch_amg_restrict(const Sell& R, const PcgState* st, const double* x, const double* x2, const double* dinv_c,
                         double omega_c, double* b_c, double* x_c, hipStream_t s);
// x_new = x_old + P x_c (x_new may alias x_old)
void launch_amg_prolong(const Sell& P, const PcgState* st, const double* x_c, const double* x_old, double* x_new,
                        hipStream_t s);
// y = x + omega dinv (b - A x)
void launch_amg_post(const Sell& A, const PcgState* st, const double* x, const double* b, const double* dinv,
                     double omega, double* y, hipStream_t s);
// z = x0 + P x_c, (z.z, z.r) records and the reduction tail; returns the record count
int launch_amg_prolong0(const Sell& P, const PcgState* st, const double* x_c, const double* x0, const double* r,
                        double* z, double* partials, const RedTail* tail, hipStream_t s);
// the fine cell operator V = M + dt alpha K of an unstructured mesh, SELL-64
// (device pointers of tv_um.hip's setup)
Sell um_operator(const UmGrid& g);

struct UmDevice;  // device allocations of one unstructured mesh (tv_um.hip)
// builds the operators on the device (stream s, synchronised before return)
int um_setup(int dim, int64_t nv, int64_t nrow, const double* xyz, int64_t nc, const int64_t* cells, UmGrid& g,
             UmDevice*& dev, hipStream_t s, std::string& err);
// halo of a partitioned unstructured mesh: out[k] = v[idx[k]], k < n (pack of
// the owned values every neighbour holds as ghosts)
void launch_um_pack(const int64_t* idx, int64_t n, const double* v, double* out, hipStream_t s);
void um_free(UmDevice* dev);
int64_t um_boundary_vertices(const UmDevice* dev, std::vector<unsigned char>& mask);  // host mask, returns count
int64_t um_nnz(const UmDevice* dev);                       // stored entries incl. SELL padding
int um_num_blocks(const UmGrid& g);                        // partial records of the fused launch
int um_rcb(int dim, int64_t nv, const double* xyz, int64_t nc, const int64_t* cells, int n_parts, int* part,
           std::string& err);
void launch_um_residual(const UmGrid& g, const double* T, const double* Tp, double* F, hipStream_t s);
void launch_um_japply(const UmGrid& g, const double* T, const double* x, double* y, hipStream_t s);
// The level-0 transfers of the geometric hierarchy (tv_amg.cpp geometric_p) on
// a structured grid of fn[0] x fn[1] x fn[2] vertices, its coarse grid cn[],
// applied by index arithmetic (no stored matrix): b_c = P^T r, x_c = omega_c
// dinv_c b_c; and z = x0 + P x_c with the (z.z, z.r) records and the KSPCG
// tail (returns the record count)
void launch_geo_restrict0(const int64_t (&fn)[3], const int64_t (&cn)[3], const PcgState* st, const double* r,
                          const double* dinv_c, double omega_c, double* b_c, double* x_c, hipStream_t s);
int launch_geo_prolong0(const int64_t (&fn)[3], const int64_t (&cn)[3], const PcgState* st, const double* x_c,
                        const double* x0, const double* r, double* z, double* partials, const RedTail* tail,
                        hipStream_t s);
// a structured grid's half-stencil operator (g.J14, g.nv, g.s1, g.s2): y = A x, or
// with b != nullptr the Jacobi step y = x + omega dinv (b - A x)
void launch_sg_apply(const UmGrid& g, const PcgState* st, const double* x, const double* b, const double* dinv,
                     double omega, double* y, hipStream_t s);
// J14 <- V14 + the Robin facet Jacobian at T (structured topology; a no-op else):
// before the J x launches of a Newton iteration (J(T) is fixed inside a solve)
void launch_um_robin_fold(const UmGrid& g, const double* T, hipStream_t s);
void launch_um_diag(const UmGrid& g, const double* T, double* d, int invert, hipStream_t s);
// p <- z + beta p (iteration it_host's parity buffer), w <- J p, p.w; the
// reduction tail (rt.counter != nullptr) reduces the records and runs the
// logic.  Returns the number of partial records.
int launch_um_japply_fused(const UmGrid& g, const double* T, const double* z, double* pA, double* pB, double* w,
                           const PcgState* st, double* partials, int it_host, const RedTail* tail, hipStream_t s);

// ---- kernel launchers (tv_cg.hip, tv_dg.hip, tv_visco.hip, tv_pcg.hip) ----
void launch_cg_residual(const CgGrid& g, const double* T, const double* Tp, double* F, hipStream_t s);
// the residual plus the boundary rows of dinv = 1 / diag J(T) in its boundary
// pass (3D marching path; the T-independent interior of dinv must already be
// in place).  Returns false (nothing launched) where that path does not apply.
bool launch_cg_residual_diag(const CgGrid& g, const double* T, const double* Tp, double* F, double* dinv,
                             hipStream_t s);
void launch_cg_japply(const CgGrid& g, const double* T, const double* x, double* y, double* partials,
                      int* n_partials, hipStream_t s, const PcgState* st = nullptr);
// returns true when the launch ends with the in-kernel reduction tail (the
// caller then skips the separate reduce launch)
// it_host: the PCG iteration index the host launches (== st->it while the
// solve runs), selects the p buffer pair without a dependent device load
bool launch_cg_japply_fused(const CgGrid& g, const double* T, const double* z, double* pA, double* pB,
                            double* w, const PcgState* st, double* partials, int* n_partials,
                            hipStream_t s, const RedTail* tail = nullptr, int it_host = 0);
// Vectors of the single-reduction PCG iteration (k_cgs_march, tv_cg.hip); the
// in / out pairs are the two parities of ping-pong buffers.
struct CgsBuffers {
  const double* T;     // temperature (facet terms)
  const double* rin;   // r_{i-1} (i = 1: the Newton residual F; INIT: r_0 = F)
  double* rout;        // r_i
  const double* sin;   // s_{i-2}
  double* sout;        // s_{i-1}
  const double* win;   // w_{i-1} without the face-workgroup facet terms
  double* wout;        // w_i (march part)
  const double* fin;   // facet terms f_{i-1} (CgGrid::ffbuf layout)
  double* fout;        // f_i
  double* p;           // p (owned nodes, in place)
  double* x;           // dx (owned nodes, in place)
  const double* dinv;  // B = diag(J)^-1
};

// One single-reduction PCG iteration (Chronopoulos-Gear CG) fused with the
// marching Jacobian, 3D CG1 path only (cg_cgs_supported): init = iteration 0
// (z_0 = B r_0, w_0 = J z_0, x = 0); tail->kind 4 / 5 runs the logic in the
// tail, or lag_sums != nullptr (multi-rank) makes every workgroup apply the
// logic of the previous iteration's all-reduced sums first.  Records: width 3,
// cg_cgs_records of them.
bool launch_cg_cgs(const CgGrid& g, bool init, const CgsBuffers& v, PcgState* st, double* partials,
                   hipStream_t s, const RedTail* tail, int it_host, const double* lag_sums);
int cg_cgs_records(const CgGrid& g);
bool cg_cgs_supported(const CgGrid& g);
// bnd_only: only the physical-boundary nodes (3D marching path; the interior of
// dinv, T-independent, is already in place from an earlier call with the same invert)
void launch_cg_diag(const CgGrid& g, const double* T, double* dinv, int invert, hipStream_t s, bool bnd_only = false);
int cg_num_blocks(const CgGrid& g, bool with_ghost_planes);

void launch_dg_residual(const DgGrid& g, const double* T, const double* Tp, double* F, hipStream_t s);
// st: queued multigrid work exits once the solve has converged (3D tiles)
void launch_dg_japply(const DgGrid& g, const double* T, const double* x, double* y, double* partials,
                      int* n_partials, hipStream_t s, const PcgState* st = nullptr);
// 3D: k_dg_tile, with the reduction tail when `tail` is given (returns true)
bool launch_dg_japply_fused(const DgGrid& g, const double* T, const double* z, double* pA, double* pB,
                            double* w, const PcgState* st, double* partials, int* n_partials,
                            hipStream_t s, const RedTail* tail = nullptr);
void launch_dg_diag(const DgGrid& g, const double* T, double* dinv, int invert, hipStream_t s);
int dg_num_blocks(const DgGrid& g);  // partial records of the largest DG launch
// cell-block Jacobi of 3D DG1 (the multigrid smoother), applied by fast
// diagonalisation of the 8 x 8 cell blocks of J(T); gface = per boundary facet
// mean of dg(T) (dg_gface_size doubles, refreshed per Newton iteration)
int64_t dg_gface_size(const DgGrid& g);
void launch_dg_gface(const DgGrid& g, const double* T, double* gface, hipStream_t s);
// mode 0: x <- omega B^-1 b ; mode 1: x <- x + omega B^-1 (b - w)
void launch_dg_bsmooth(const DgGrid& g, const PcgState* st, const double* b, const double* w, const double* gface,
                       double omega, double* x, int mode, hipStream_t s);
// r <- r - a w, x0 <- omega B^-1 r, dx moved every second iteration from iteration 1 on
// (init: x0 <- omega B^-1 r only; launch_mg_dx_finish ends the solve)
void launch_dg_bupdate(const DgGrid& g, const PcgState* st, const double* pA, const double* pB, const double* w,
                       const double* gface, double omega, double* r, double* dx, double* x0, int it_host, int init,
                       hipStream_t s);
// z <- x0 + omega B^-1 (r - w), (z.z, z.r) records + reduction tail; returns the record count
int launch_dg_bpost(const DgGrid& g, const PcgState* st, const double* x0, const double* r, const double* w,
                    const double* gface, double omega, double* z, double* partials, const RedTail* tail, hipStream_t s);

void launch_visco(int dim, int all, const ViscoConst& c, const ViscoFields& f, hipStream_t s);
void launch_visco_Tpass(int dim, int all, const ViscoConst& c, const ViscoFields& f, hipStream_t s);
void launch_visco_Spass(int dim, int all, const ViscoConst& c, const ViscoFields& f, hipStream_t s);

// PCG vector kernels over the owned range [0, n) of already-offset pointers
constexpr int kVecBlocks = 1024;        // grid cap of the vector kernels
constexpr int kVecBlocksMin = 256;      // below this the grid no longer shrinks with n
constexpr int kVecNodesPerThread = 16;
constexpr int kVecBlocksMax = 8192;  // partial-record capacity of the vector kernels
void launch_pcg_init(int64_t n, const double* r, const double* dinv, double* z, double* dx,
                     double* partials, hipStream_t s);
// PCG update of iteration it_host: w += facet terms, r <- r - a w, z <- B r
// with r = z / dinv (r is not stored: its recurrence runs through z), and on
// odd iterations dx <- dx + a_prev p_prev + a p (both p buffers are live, so
// the dx stream is read and written every second iteration only); p is taken
// from buffer (it_host & 1 ? pB : pA), matching the fused matvec
// Robin facet terms the fused CG matvec leaves out of w (marching path): the
// PCG update adds fface at the owned boundary nodes (see k_cg_march)
struct FaceAdd {
  int on;
  int n0, n1, n2;
  int64_t t_off;             // local index of the first owned node
  double inv_n0, inv_plane;  // 1/n0, 1/(n0 n1) (index -> coordinates)
  const double* ff[6];
};
FaceAdd cg_face_add(const CgGrid& g, int64_t t_off);


// ---- geometric multigrid on the box hierarchy (tv_mg.hip, tv_pcg.hip) ----
// Transfer between a level and the next coarser one (nested rectilinear grids:
// along a coarsened axis fine node 2I is coarse node I, odd fine nodes
// interpolate linearly between their two coarse neighbours).  Per storage
// axis: prolongation = two (coarse index, weight) pairs per fine node,
// restriction (its transpose) = three (fine index, weight) pairs per coarse
// node; indices are local (ghost planes included).
struct MgXfer {
  int fn[3], cn[3];           // local node counts of the fine / coarse level
  int coarse[3];              // axis coarsened (else identity along it)
  int f_kb, f_ke, c_kb, c_ke; // owned planes (storage axis 2) of the fine / coarse level
  const int* pi[3];           // [2 fn[a]]
  const double* pw[3];
  const int* ri[3];           // [3 cn[a]]
  const double* rw[3];
  // 1: fine local plane 2K + b interpolates from coarse local planes K, K + 1
  // along axis 2 (both levels whole boxes: the 2 x 2 block prolongation
  // applies); 0 on a partitioned level, whose local planes start anywhere
  int aligned;
};
// bc <- P^T (bf - (wf + facet terms fa)) on the coarse owned nodes (mask:
// level-0 dinv, 0 = excluded node); xc != nullptr: also the coarse level's
// pre-smoothing from 0, xc <- omega_c dinv_c bc
void launch_mg_restrict(const MgXfer& x, const PcgState* st, const double* bf, const double* wf, const FaceAdd* fa,
                        const double* mask, double* bc, const double* dinv_c, double omega_c, double* xc,
                        hipStream_t s);
// Fused residual restriction (tv_mg.hip k_mg_rrestrict): b_c = R (b - J x) on a
// rectilinear level WITHOUT forming J x.  On the box R = Rq (x) Rr (x) Rx and J
// is a sum of Kronecker products of the 1D mass / stiffness rows, so R J is a
// sum of Kronecker products of the per-axis operators (R_a M_a), (R_a K_a):
// five fine nodes wide per coarse node, applied by sum factorisation (x in the
// lanes, the row axis over five fine rows per wave, the march axis over a
// sliding five-plane window).  The Robin facet part of J x comes from
// k_cg_facet_faces (fface of all six faces), subtracted from b on the face nodes.
struct RRAxis {
  const int* f0;     // [cn]: first fine node of coarse node I's window (its fine node - 2)
  const double* w;   // [cn][15]: (R M), (R K), R over fine nodes f0 .. f0 + 4 (0 outside the axis)
};
struct RRArgs {
  int on;
  int fn[3], cn[3];
  RRAxis ax[3];
  double da;           // dt alpha
  int raxis, nseg, qchunk;
};
void launch_mg_rrestrict(const RRArgs& a, const PcgState* st, const double* b, const double* x, const FaceAdd& fa,
                         double* bc, const double* dinv_c, double omega_c, double* xc, hipStream_t s);
void launch_cg_facet_faces(const CgGrid& g, const double* T, const double* x, const PcgState* st, hipStream_t s);
FaceAdd cg_face_add_all(const CgGrid& g);  // the facet terms of every physical face (fface[] of g)

// The coarse level's post-smoothing operands: the prolongation applies
// xc + omega dinv (b - (w + facet terms fa)) instead of xc
struct CoarsePost {
  const double* b;
  const double* w;
  const double* dinv;
  double omega;
  FaceAdd fa;
};
// xf <- xf + P xc on the fine owned nodes (mask as above: x stays 0 on excluded nodes);
// cp != nullptr: the smoothed xc (only where mg_prolong_smooths(x))
void launch_mg_prolong(const MgXfer& x, const PcgState* st, double* xf, const double* xc, const double* mask,
                       hipStream_t s, const CoarsePost* cp = nullptr);
bool mg_prolong_smooths(const MgXfer& x);
// launch_mg_restrict adds the facet terms of a FaceAdd itself (else the caller
// must hand it a complete J x)
bool mg_restrict_folds_faces(const MgXfer& x);
// mode 0: x <- omega dinv b ; mode 1: x <- x + omega dinv (b - (w + facet terms fa))    (damped Jacobi)
void launch_mg_jacobi(int64_t n, const PcgState* st, const double* b, const double* w, const FaceAdd* fa,
                      const double* dinv, double omega, double* x, int mode, hipStream_t s);
void launch_mg_inject(const MgXfer& x, const double* Tf, double* Tc, hipStream_t s);  // coarse T <- fine T
// the same on the coarse local planes [k0, k1) only
void launch_mg_inject_range(const MgXfer& x, const double* Tf, double* Tc, int k0, int k1, hipStream_t s);
// w <- b - (w + facet terms fa) on n nodes (0 where mask == 0): the residual a
// partitioned level exchanges and restricts
void launch_mg_resid(int64_t n, const PcgState* st, const double* b, double* w, const FaceAdd* fa, const double* mask,
                     hipStream_t s);
// mask <- 1 on the local nodes [own0, own1) where dinv != 0 (dinv may be null), else 0
void launch_mg_ownmask(int64_t n, int64_t own0, int64_t own1, const double* dinv, double* mask, hipStream_t s);
// Per-Newton preparation of up to kMgPrepMax coarse CG levels in two launches
// (instead of an injection and a boundary-diagonal launch per level): T of
// every level injected straight from the base level's T through the composed
// index maps, then the boundary rows of every level's dinv (the
// T-independent interiors must already be in place)
constexpr int kMgPrepMax = 4;  // keeps the kernel argument block near 2 KB
struct MgPrep {
  int nlev;
  const double* Tbase;            // T of the level the first transfer starts from
  MgXfer xf[kMgPrepMax];          // level i's transfer from level i - 1 (i = 0: from the base)
  double* T[kMgPrepMax];
  double* dinv[kMgPrepMax];
  CgGrid g[kMgPrepMax];
  int64_t off_n[kMgPrepMax + 1];  // 64-padded offsets of the levels' nodes / boundary nodes
  int64_t off_b[kMgPrepMax + 1];
};
void launch_mg_prepare(const MgPrep& p, hipStream_t s);
bool cg_uses_march(const CgGrid& g);  // the 3D marching kernels (not the x-row kernel) serve this grid
// DG1 level 0 -> CG1 level 1 of the same box (3D; DG dofs as DgGrid lays them
// out, l = a + 2b + 4c over the storage axes): restriction = sum of the
// cell-local copies at each vertex (P = injection of the vertex value into
// every copy), with the CG level's pre-smoothing fused when xc is given (one
// partition).  A slab writes its vertex planes of the global CG vector (kg0 =
// global layer of its local layer 0): the restriction from its owned cells,
// the prolongation into every local cell (ghost layers included), the vertex
// mean of T on its owned vertex planes
void launch_mg_dg_restrict(const DgGrid& g, const PcgState* st, const double* bf, const double* wf, const double* mask,
                           double* bc, const double* dinv_c, double omega_c, double* xc, int kg0, hipStream_t s);
void launch_mg_dg_prolong(const DgGrid& g, const PcgState* st, double* xf, const double* xc, const double* mask,
                          int kg0, hipStream_t s);
void launch_mg_dg_T(const DgGrid& g, const double* Tdg, double* Tcg, int kg0, hipStream_t s);  // vertex mean
// power-iteration step for lambda_max(D^-1 J): y <- dinv .* y, per-block sums of y^2 (returns the count)
int launch_mg_pow(int64_t n, const double* dinv, double* y, double* partials, hipStream_t s);
void launch_mg_scale(int64_t n, const double* y, double a, double* x, hipStream_t s);  // x <- a y
// complete J x with x.(J x) reduced by the tail (kind 0: into tail->out[0]);
// false where the marching kernel does not serve the grid (no tail ran)
bool launch_cg_japply_tail(const CgGrid& g, const double* T, const double* x, double* y, const PcgState* st,
                           double* partials, const RedTail* tail, hipStream_t s);
// J x without the facet terms of the faces along the march (the FaceAdd the
// consumer adds, cg_face_add); the whole J x where the row kernel runs
void launch_cg_japply_partial(const CgGrid& g, const double* T, const double* x, double* y, const PcgState* st,
                              hipStream_t s);
// level 0 of the PCG (tv_pcg.hip): r <- r - a (w + facet terms), dx <- dx + a p,
// x0 <- omega dinv r (the V-cycle's pre-smoothing from 0); init: x0 <- omega dinv r (dx is
// assigned by iteration 1 / launch_mg_dx_finish)
void launch_mg_update(int64_t n, const PcgState* st, const double* pA, const double* pB, const double* w,
                      const FaceAdd* fa, const double* dinv, double omega, double* r, double* dx, double* x0,
                      int it_host, int init, hipStream_t s, const double* lag = nullptr,
                      unsigned* counter = nullptr);
// the single-reduction form's update (k_mg_update_cgs, tv_pcg.hip): s <- u + beta s,
// p <- z + beta p, dx <- dx + a p, r <- r - a s, x0 <- omega dinv r (first: s = u,
// p = z, dx = a p); lag: the all-reduced sums whose logic (lag_kind 6 / 7) this
// launch forms and its last workgroup (counter) commits
void launch_mg_update_cgs(int64_t n, const PcgState* st, const double* u, double* s, const double* z, double* p,
                          double* dx, double* r, const double* dinv, double omega, double* x0, bool first,
                          const double* lag, int lag_kind, unsigned* counter, hipStream_t stream);
// the same post-smoothing fused into the level-0 J x march (k_cg_march POST)
// plus a pass over the side-face nodes for the face-workgroup facet terms
// (k_mg_post_faces, which runs the reduction tail); z <- x + omega dinv (r - J x),
// w untouched.  Returns the record count, or -1 where the march path does not
// apply (the caller then runs J x + launch_mg_post)
int launch_cg_japply_post(const CgGrid& g, const double* T, const double* x, const double* r, const double* dinv,
                          double omega, double* z, const PcgState* st, double* partials, const RedTail* tail,
                          hipStream_t s);
// z <- x0 + omega dinv (r - (w + facet terms)) (post-smoothing), (z.z, z.r) records + reduction tail;
// returns the record count
int launch_mg_post(int64_t n, const PcgState* st, const double* x0, const double* r, const double* w,
                   const FaceAdd* fa, const double* dinv, double omega, double* z, double* partials,
                   const RedTail* tail, hipStream_t s);

void launch_pcg_update(int64_t n, PcgState* st, const double* pA, const double* pB, const double* w,
                       const double* dinv, double* dx, double* z, double* partials, hipStream_t s,
                       const RedTail* tail = nullptr, const FaceAdd* fa = nullptr, int it_host = 0);
// after a solve of `its` iterations with its odd: dx <- dx + a p of the last
// iteration (the step the pairwise dx update has not applied yet)
void launch_pcg_dx_tail(int64_t n, const PcgState* st, const double* pA, const double* pB, double* dx, int its,
                        hipStream_t s);
// end of a multigrid solve (k_mg_update leaves dx unset until iteration 1
// assigns it): its 0 -> dx = 0, its 1 -> dx = a p, else launch_pcg_dx_tail
void launch_mg_dx_finish(int64_t n, const PcgState* st, const double* pA, const double* pB, double* dx, int its,
                         hipStream_t s);
// one-block deterministic reduce of n records of width W (<= 2) into out[W];
// kind: 0 none, 1 PCG init logic, 2 PCG p.w logic, 3 PCG update logic
void launch_reduce_logic(const double* partials, int n, int W, double* out, PcgState* st, int kind,
                         int check_done, hipStream_t s);
void launch_logic(PcgState* st, const double* sums, int kind, hipStream_t s);
// gate: a Newton decision word (k_newton_test); nonzero -> the solve is marked
// done with R_SKIPPED, so every launch queued behind it exits at once
void launch_set_state(PcgState* st, const PcgState& h, hipStream_t s, const double* gate = nullptr);
// T <- T - dx, ||dx||^2 partials; with `tail` the last workgroup reduces them into tail->out
void launch_newton_update(int64_t n, double* T, const double* dx, double* partials, hipStream_t s,
                          const RedTail* tail = nullptr);
// the post-solve group of a Newton iteration, gated on the solver state (runs
// once, behind the batch that ends the solve): dx finish, T <- T - dx, ||dx||^2
// into sums[0] (single partition); pA == nullptr: the single-reduction form (dx complete)
void launch_post_group(int64_t n, const PcgState* st, const double* pA, const double* pB, double* dx, double* T,
                       double* partials, double* sums, hipStream_t s);
int pcg_vec_blocks(int64_t n);
void launch_fill(double* x, int64_t n, double v, hipStream_t s);

// ---- time-series output (tv_output.cpp) ----
struct Output;
Output* output_create(const std::string& dir, int dim, const std::vector<std::vector<double>>& Xs, const int* phys,
                      std::string& err);
Output* output_create_unstructured(const std::string& dir, int dim, const std::vector<double>& xyz,
                                   const std::vector<int64_t>& cells, std::string& err);
bool output_add_field(Output* o, const std::string& name, int ncomp, bool dg, size_t n_values, std::string& err);
bool output_start(Output* o, int device, std::string& err);
double* output_acquire(Output* o, int* set);
size_t output_offset(const Output* o, size_t k);
void output_release(Output* o, int set);  // an acquired set whose write is abandoned
bool output_submit(Output* o, int set, double t, hipStream_t compute, std::string& err);
std::string output_destroy(Output* o);
void launch_copy(double* dst, const double* src, int64_t n, hipStream_t s);
// the same, gated on the Newton test (tv_visco.hip)
void launch_copy_gated(double* dst, const double* src, int64_t n, const NewtonGate& g, hipStream_t s);

}  // namespace tv
