/*
 * tvfem.h — C-ABI of libtvfem.so, the MI355X (gfx950) native hot path of the
 * thermo-viscoelastic glass-tempering solver (pzimbrod/fem-glass-tempering).
 *
 * Plain C types only (no torch, no HIP types in any signature).  One opaque
 * context per GPU / per mesh partition.  Every function returns an int status
 * (TV_OK = 0); the message of the last failure is available through
 * tv_last_error(ctx) (or tv_last_error(NULL) for failures before a context
 * exists).  All device work is stream-ordered on the context's HIP stream.
 *
 * What each entry point replaces in the reference (file:line under
 * /root/reference; [3P] = third-party code the reference drives):
 *
 *   tv_create            ThermoViscoProblem.__init__ (ThermoViscoProblem.py:24-58):
 *                        mesh read (:27-28), spaces (:61-103), functions
 *                        (:106-173), ThermalModel/ViscoelasticModel constants
 *                        (ThermalModel.py:7-29, ViscoelasticModel.py:10-84).
 *   tv_set_initial_condition  _set_initial_condition (ThermoViscoProblem.py:187-233).
 *   tv_set_field / tv_get_field  Function.x.array reads/writes of the state dicts
 *                        functions/functions_current/_previous/_next (:112-171),
 *                        in the reference's interleaved blocked layout
 *                        x.array[dof*bs + comp].
 *   tv_residual          NonlinearProblem.F -> dolfinx assemble_vector over the
 *                        FFCx cell / exterior-facet / interior-facet kernels of
 *                        the form at ThermoViscoProblem.py:293-325 [3P].
 *   tv_jacobian_apply    NonlinearProblem.J (ufl.derivative of F, :331) assembled
 *                        by dolfinx assemble_matrix [3P] and applied by PETSc
 *                        MatMult inside KSPSolve — here matrix-free.
 *   tv_jacobian_diag     PETSc MatGetDiagonal (PC setup) [3P].
 *   tv_precond_apply     PCApply of the KSP's preconditioner (PCGAMG, :343-346)
 *                        [3P]: Jacobi, or one geometric-multigrid V-cycle.
 *   tv_solve_T           _solve_T (:384-391): dolfinx NewtonSolver.solve
 *                        (incremental criterion, rtol 1e-12, :334-337) with
 *                        KSP cg (:343) — Jacobi-PCG instead of GAMG (:344).
 *   tv_visco_update      _solve_Tf/_solve_strains/_solve_shifted_time/_solve_stress
 *                        (:393-595): the 17 fem::interpolate(Expression) passes
 *                        of ViscoelasticModel._init_expressions
 *                        (ViscoelasticModel.py:86-242), fused into one pass.
 *   tv_step              solve_timestep (:367-381) minus the file output (:374).
 *   tv_comm_*            MPI COMM_WORLD + dolfinx Scatterer::scatter_forward
 *                        (:351) + PETSc VecNorm/VecDot MPI_Allreduce [3P],
 *                        replaced by RCCL over xGMI.
 */
#ifndef TVFEM_H
#define TVFEM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TV_ABI_VERSION 8  /* 2: tv_options gained pcg_variant, model_mode, preconditioner, mg_levels;
                            3: dg_kernel, dg_tile_chunk, mg_replicate_nodes, ksp_fixed_its;
                            4: tv_upart_desc / tv_create_unstructured_part;
                            5: tv_comm_init_loopback, tv_comm_check, tv_options.mg_coupling;
                            6: tv_comm_time;
                            7: tv_get_options, tv_set_newton_tolerances, tv_set_ksp_tolerances,
                               tv_last_converged;
                            8: tv_options lost the unused use_graphs field */

/* status codes */
#define TV_OK 0
#define TV_ERR_ARG 1          /* invalid argument */
#define TV_ERR_HIP 2          /* HIP runtime failure */
#define TV_ERR_NOT_CONVERGED 3 /* Newton did not converge (dolfinx raises) */
#define TV_ERR_KSP 4          /* Krylov solver diverged */
#define TV_ERR_STATE 5        /* field not available in this mode */
#define TV_ERR_COMM 6         /* RCCL failure */

/* finite element families (ThermoViscoProblem.py:70-71 allows CG and DG) */
#define TV_CG 0
#define TV_DG 1

/* Mesh: rectilinear grid (tensor product of per-axis node coordinates).  Covers
 * the reference's 1D interval meshes (geometry.py, any node spacing) and the
 * structured 3D hexahedral plates of the benchmark configurations.
 *   dim             topological dimension 1..3
 *   n_cells[a]      cells along physical axis a (a < dim)
 *   coords[a]       n_cells[a]+1 increasing node coordinates along axis a
 *   part_axis       physical axis along which the mesh is sliced into
 *                   partitions (-1: automatic = longest of the axes >= 1)
 *   n_parts, part   number of partitions / this context's partition
 * A partition (dim >= 2) is a slab: CG T owns node planes with one ghost plane
 * per interface, DG T owns cell layers with one ghost cell layer; mixed
 * families (DG T / CG sigma as main.py, or CG T / DG sigma) partition the T
 * space so and give sigma the owned nodes / cells it reads from it
 * (tv_num_dofs returns each space's owned count and global offset). */
typedef struct {
  int dim;
  int n_cells[3];
  const double* coords[3];
  int part_axis;
  int n_parts;
  int part;
} tv_mesh_desc;

/* Unstructured mesh: quadrilaterals (dim 2) or hexahedra (dim 3) of any
 * shape, as gmsh writes them (geometry.py / gmshio.read_from_msh at
 * ThermoViscoProblem.py:27-28).  coords: 3 doubles per vertex; cells: 2^dim
 * vertex ids per cell in the tensor local order l = a + 2b + 4c (basix /
 * dolfinx order).  CG1 temperature and stress spaces; assembled by the
 * element-local kernels (csrc/tv_um.hip). */
typedef struct {
  int dim;
  int64_t n_vertices;
  const double* coords;
  int64_t n_cells;
  const int64_t* cells;
} tv_umesh_desc;

/* One partition of a distributed unstructured mesh (the dolfinx mesh
 * distribution of gmshio.read_from_msh(..., MPI.COMM_WORLD, 0) at
 * ThermoViscoProblem.py:27-28, with the ghost layer dolfinx keeps for the
 * scatter_forward of :351).  The local tv_umesh_desc passed with it holds
 *   vertices: the n_owned owned vertices first, then the ghosts grouped by
 *             owner in the order of `neighbors` (recv_count[k] of them for
 *             neighbors[k]), each group in the owner's send order;
 *   cells:    the n_owned_cells cells of this part first, then every other
 *             cell that touches an owned vertex (so each owned row of F and J
 *             is complete).
 * The halo sends send_count[k] owned values, at the local indices listed in
 * send_idx (concatenated over k), to neighbors[k] and receives that
 * neighbour's ghosts in place.  global_offset: global index of owned vertex 0
 * in the partition-major numbering (sum of the lower parts' n_owned). */
typedef struct {
  int n_parts;
  int part;
  int64_t n_owned;
  int64_t n_owned_cells;
  int64_t global_offset;
  int n_neighbors;
  const int* neighbors;        /* ascending ranks */
  const int64_t* recv_count;   /* n_neighbors */
  const int64_t* send_count;   /* n_neighbors */
  const int64_t* send_idx;     /* sum(send_count) local owned indices */
} tv_upart_desc;

typedef struct {
  int T_family;      /* TV_CG / TV_DG  (fe_config["T"]["element"])      */
  int T_degree;      /* must be 1                                        */
  int sigma_family;  /* TV_CG / TV_DG  (fe_config["sigma"]["element"])  */
  int sigma_degree;  /* must be 1                                        */
} tv_fe_config;

/* model_params of main.py:29-55 plus the Prony tableaux of
 * ViscoelasticModel.py:19-68 (6 terms each).  rho, cp, k and Tf_init are
 * accepted and unused, exactly as in the reference. */
typedef struct {
  double f, epsilon, sigma, T_ambient, T_0, alpha, htc, rho, cp, k;
  double H, Tb, Rg, alpha_solid, alpha_liquid, Tf_init;
  double m_n[6], lambda_m[6], g_n[6], lambda_g[6], k_n[6], lambda_k[6];
  double dt;
} tv_params;

/* Solver options.  Defaults (tv_default_options): dolfinx NewtonSolver
 * (rtol 1e-12 set at ThermoViscoProblem.py:336; atol 1e-10, max_it 50,
 * relaxation 1 [3P defaults]) and PETSc KSP (rtol 1e-5, atol 1e-50,
 * dtol 1e5, max_it 10000 [3P defaults]). */
typedef struct {
  double newton_rtol, newton_atol;
  int newton_max_it;
  int error_on_nonconvergence;
  double ksp_rtol, ksp_atol, ksp_dtol;
  int ksp_max_it;
  int materialize;        /* 0: state fields only, 1: every reference field  */
  int pcg_batch;          /* iterations launched between convergence polls  */
  int pcg_variant;        /* TV_PCG_AUTO / TV_PCG_KSPCG / TV_PCG_SINGLE_REDUCTION */
  int model_mode;         /* TV_MODEL_REFERENCE (default) / TV_MODEL_PAPER       */
  int preconditioner;     /* TV_PC_JACOBI (default) / TV_PC_GMG (box meshes) /
                             TV_PC_AMG (unstructured meshes, one partition)      */
  int mg_levels;          /* GMG: levels incl. the fine one (0: automatic)       */
  int dg_kernel;          /* 3D DG1 Jacobian: TV_DG_KERNEL_AUTO / _TILE / _CELLS */
  int dg_tile_chunk;      /* planes per marching DG tile (0: automatic = 5)      */
  int mg_replicate_nodes; /* partitioned GMG: coarse levels of at most this many
                             nodes are replicated on every rank (0: 300000)     */
  int ksp_fixed_its;      /* > 0: every Krylov solve runs exactly this many
                             iterations, with no convergence test (PETSc
                             KSP_NORM_NONE + max_it; timing of partition shares
                             with the communication stubbed); tv_step then ends
                             every step (visco update) whatever the Newton test */
  int mg_coupling;        /* partitioned GMG: TV_MG_COUPLING_AUTO / _GLOBAL / _LOCAL */
} tv_options;

/* Coupling of the partitioned geometric multigrid (the Krylov iteration is
 * always global: matvec over the ghost planes, all-reduced dot products):
 *   GLOBAL  the V-cycle of the whole box, distributed (ghost planes of every
 *           level exchanged, the small coarse levels replicated): the same
 *           preconditioner as on one partition, ~5 exchanges per V-cycle;
 *   LOCAL   block Jacobi over the partitions: each partition runs the V-cycle
 *           of its own slab (the hierarchy of its owned planes, zero values
 *           beyond them: the principal block of the operator) -- no exchange
 *           inside the preconditioner, 2 exchange points per Krylov iteration.
 *           The Krylov counts then depend on the partition count, as PCGAMG's
 *           (its smoothers and coarse solve are process-local) do: ~2.4x the
 *           GLOBAL count at C4's cell sizes (tools/mg_coupling_model.py);
 *   AUTO    GLOBAL. */
#define TV_MG_COUPLING_AUTO 0
#define TV_MG_COUPLING_GLOBAL 1
#define TV_MG_COUPLING_LOCAL 2

/* 3D DG1 Jacobian kernel: AUTO = TILE, the marching tile kernel (production);
 * CELLS = one thread per cell, the straightforward SIPG evaluation the tile
 * kernel is checked against (tests/test_gpu_parity.py). */
#define TV_DG_KERNEL_AUTO 0
#define TV_DG_KERNEL_TILE 1
#define TV_DG_KERNEL_CELLS 2

/* Preconditioner of the Krylov solve (the reference configures PCGAMG,
 * ThermoViscoProblem.py:343-346; PETSc's GAMG is not reproducible here):
 *   JACOBI  point Jacobi (the oracle's PETSc KSPCG + PCJACOBI restatement; the
 *           Krylov iteration counts the parity tests compare);
 *   GMG     geometric multigrid V-cycle on the box hierarchy (3D CG1 and DG1
 *           rectilinear meshes, one partition or slabs): the box coarsened by two
 *           along every axis with an even cell count until the coarsest level
 *           is mass-dominated (dt alpha / h^2 <= 0.5) or cannot coarsen, damped
 *           Jacobi smoothing (Gershgorin-bounded weight), coarse operators
 *           re-discretised with T injected.  Same Newton solution (the linear
 *           solves reach the same relative tolerance), ~4 instead of ~33 Krylov
 *           iterations per solve at C4. */
#define TV_PC_JACOBI 0
#define TV_PC_GMG 1
#define TV_PC_AMG 2   /* algebraic multigrid (csrc/tv_amg.cpp), the PCGAMG of ThermoViscoProblem.py:344:
                         smoothed aggregation; on a mesh with structured topology
                         (one partition) index-space geometric transfers with
                         Galerkin coarse operators */

/* Model semantics.  REFERENCE reproduces the reference as it runs, quirks
 * included.  PAPER (opt-in, never the default) applies
 * the fixes the reference's comments name: Eq. 25 drives the partial fictive
 * temperatures (ViscoelasticModel.py:100-108), Tf_prev is updated after the
 * thermal strain (ThermoViscoProblem.py:481 vs :492), xi takes the trapezoidal
 * "+" (ViscoelasticModel.py:171), s~ / sigma~ are fed from the previous s /
 * sigma partial stresses (Eq. 16, ViscoelasticModel.py:195-209), and a
 * Dirichlet condition can be applied (tv_set_dirichlet). */
#define TV_MODEL_REFERENCE 0
#define TV_MODEL_PAPER 1

/* Krylov iteration form (same Jacobi-PCG iterates in exact arithmetic):
 *   KSPCG             PETSc KSPSolve_CG as written: two reductions per iteration
 *                     (p.w, then z.z and z.r), a fused matvec and an update launch;
 *   SINGLE_REDUCTION  Chronopoulos-Gear form: one launch and one reduction per
 *                     iteration (3D CG1 temperature only);
 *   AUTO              SINGLE_REDUCTION (Jacobi) on 3D CG1 box meshes partitioned
 *                     into slabs of <= 3M owned nodes (one communication round
 *                     per iteration) or on one partition of <= 1.5M nodes (one
 *                     launch per iteration), else KSPCG.  With TV_PC_GMG on a
 *                     slab partition AUTO selects the single-reduction GMG-PCG
 *                     (deep-ghost slabs); an explicit SINGLE_REDUCTION is the
 *                     Jacobi form only and is refused with TV_PC_GMG. */
#define TV_PCG_AUTO 0
#define TV_PCG_KSPCG 1
#define TV_PCG_SINGLE_REDUCTION 2

/* field ids (the reference's Function objects) */
enum {
  TV_F_T = 0,               /* functions_current["T"]                        */
  TV_F_T_PREV,              /* functions_previous["T"]                       */
  TV_F_T_NEXT,              /* functions_next["T"]                           */
  TV_F_TF,                  /* functions_current["Tf"]                       */
  TV_F_TF_PREV,             /* functions_previous["Tf"]                      */
  TV_F_TF_PARTIAL,          /* functions_current["Tf_partial"]   (bs 6)      */
  TV_F_TF_PARTIAL_PREV,     /* functions_previous["Tf_partial"]  (bs 6)      */
  TV_F_PHI,                 /* functions["phi"]                              */
  TV_F_PHI_NEXT,            /* functions_next["phi"]                         */
  TV_F_XI,                  /* functions["xi"]                               */
  TV_F_THERMAL_STRAIN,      /* functions["thermal_strain"]      (bs d*d)     */
  TV_F_TOTAL_STRAIN,        /* functions["total_strain"]        (bs d*d)     */
  TV_F_DEVIATORIC_STRAIN,   /* functions["deviatoric_strain"]   (bs d*d)     */
  TV_F_DS_PARTIAL,          /* functions["ds_partial"]          (bs 6*d*d)   */
  TV_F_DSIGMA_PARTIAL,      /* functions["dsigma_partial"]      (bs 6*d*d)   */
  TV_F_S_TILDE,             /* functions_current["s_tilde_partial"]          */
  TV_F_S_TILDE_NEXT,        /* functions_next["s_tilde_partial"]             */
  TV_F_SIGMA_TILDE,         /* functions_current["sigma_tilde_partial"]      */
  TV_F_SIGMA_TILDE_NEXT,    /* functions_next["sigma_tilde_partial"]         */
  TV_F_S_PARTIAL,           /* functions_current["s_partial"]                */
  TV_F_S_PARTIAL_NEXT,      /* functions_next["s_partial"]                   */
  TV_F_SIGMA_PARTIAL,       /* functions_current["sigma_partial"]            */
  TV_F_SIGMA_PARTIAL_NEXT,  /* functions_next["sigma_partial"]               */
  TV_F_SIGMA,               /* functions_next["sigma"]          (bs d*d)     */
  TV_F_RESIDUAL,            /* work: last assembled residual F               */
  TV_F_DX,                  /* work: last Newton increment dx                */
  TV_NUM_FIELDS
};

/* ---- library / context -------------------------------------------------- */
int tv_abi_version(void);
const char* tv_last_error(const void* ctx);      /* NULL ctx: global error   */
void tv_default_options(tv_options* opts);
void tv_default_params(tv_params* p);            /* main.py:29-55 + tableaux */

int tv_create(const tv_mesh_desc* mesh, const tv_fe_config* fe, const tv_params* params,
              const tv_options* opts, int device, void** ctx_out);
int tv_create_unstructured(const tv_umesh_desc* mesh, const tv_fe_config* fe, const tv_params* params,
                           const tv_options* opts, int device, void** ctx_out);
/* partition `part->part` of a distributed unstructured mesh (local mesh as
 * tv_upart_desc describes); the communicator (tv_comm_init / _host) must be
 * set before the first step (a solve without one returns TV_ERR_STATE).
 * KSPCG form with Jacobi (TV_PC_JACOBI) or the agglomerated algebraic multigrid
 * (TV_PC_AMG: at the first solve every rank gathers the GLOBAL T-independent
 * cell operator and builds the whole hierarchy -- host memory and setup time
 * per rank grow with the global nnz, O(27 x 12 B) per global vertex; refused
 * above 20M global rows, TV_ERR_ARG); Dirichlet mode as on one partition. */
int tv_create_unstructured_part(const tv_umesh_desc* local_mesh, const tv_upart_desc* part, const tv_fe_config* fe,
                                const tv_params* params, const tv_options* opts, int device, void** ctx_out);
int tv_destroy(void* ctx);

/* Host-only (no GPU needed): layout of partition `part` of a CG1 mesh with one
 * ghost plane per interface (a context with the distributed GMG keeps three on
 * its fine slab internally; the owned range is the same) —
 * out[0..2] storage axis -> physical axis (-1 degenerate), out[3..5] global
 * nodes per storage axis, out[6..7] owned node planes [b0, b1) along storage
 * axis 2, out[8] global offset of the first owned dof, out[9] owned dofs,
 * out[10] local dofs incl. ghost planes, out[11..12] ghost plane below/above. */
/* Host only (no GPU): recursive coordinate bisection of the cells of an
 * unstructured mesh into n_parts balanced parts (part_out: n_cells ids).
 * Replaces the graph partitioner dolfinx applies when it distributes the mesh
 * read at ThermoViscoProblem.py:27-28. */
int tv_partition_rcb(const tv_umesh_desc* mesh, int n_parts, int* part_out);
int tv_partition_layout(const tv_mesh_desc* mesh, int64_t* out13);

/* sizes: owned dofs of the T space / sigma space on this partition; block
 * size of a field; global dof offset of this partition's first owned dof */
int tv_num_dofs(void* ctx, int space /*0 T, 1 sigma*/, int64_t* n_owned, int64_t* global_offset);
int tv_field_block_size(void* ctx, int field, int* bs);
/* dof coordinates (owned dofs, 3 doubles each, zero-padded beyond dim) */
int tv_dof_coordinates(void* ctx, int space, double* xyz, size_t n_dofs);

/* host <-> device field transfer, owned dofs, interleaved reference layout */
int tv_set_field(void* ctx, int field, const double* host, size_t n_values);
int tv_get_field(void* ctx, int field, double* host, size_t n_values);
/* device address of a field's storage (component-major: comp*stride + dof);
 * waits for the context's queued work first (tv_step returns with the visco
 * update possibly still running on the context's stream) */
int tv_field_device_ptr(void* ctx, int field, void** dev_ptr, int64_t* comp_stride);

int tv_set_initial_condition(void* ctx, double T0);
/* Dirichlet condition T = value on every dof of the exterior boundary, applied
 * in the Newton solve as dolfinx's NonlinearProblem(bcs=...) does (lifted
 * residual, constrained dofs moved to the value by the first update):
 * _set_dirichlet_bc (ThermoViscoProblem.py:236-243) as the reference intends
 * it -- its own code cannot run (:241 self.fs, :180 material_model.T_ambient,
 * and the bc never reaches NonlinearProblem at :331).  Only with model_mode =
 * TV_MODEL_PAPER (TV_ERR_STATE otherwise).  DG temperature: no dof belongs to
 * a facet, so the constraint is empty (as locate_dofs_topological would find). */
int tv_set_dirichlet(void* ctx, int enable, double value);
int tv_sync(void* ctx);

/* Solver settings after creation: the options in force (tv_get_options), and
 * the tolerances a caller of the reference sets on problem.solver -- dolfinx
 * NewtonSolver rtol / atol / max_it / error_on_nonconvergence, the object
 * _setup_solver creates at ThermoViscoProblem.py:334-337 [3P] -- and on
 * problem.ksp = solver.krylov_solver (:339; PETSc KSPSetTolerances rtol,
 * abstol, dtol, max_it [3P]).  They take effect at the next solve;
 * TV_ERR_ARG for a negative tolerance, dtol <= 0 or max_it < 1. */
int tv_get_options(void* ctx, tv_options* out);
int tv_set_newton_tolerances(void* ctx, double rtol, double atol, int max_it, int error_on_nonconvergence);
int tv_set_ksp_tolerances(void* ctx, double rtol, double atol, double dtol, int max_it);

/* ---- operators (device pointers, owned T-dofs, length n_owned) ----------
 * The context stream is non-blocking: these calls first wait for all work
 * already queued on the device (hipDeviceSynchronize), so inputs written on
 * another stream (e.g. torch's) before the call are complete when it reads them. */
int tv_residual(void* ctx, const double* T_dev, double* F_dev);     /* F(T; T_prev) */
int tv_jacobian_apply(void* ctx, const double* x_dev, double* y_dev); /* J(T)·x      */
int tv_jacobian_diag(void* ctx, double* d_dev);                       /* diag J(T)   */
/* z = B r with the context's preconditioner at the current T (tv_options.
 * preconditioner): Jacobi z = r / diag J(T), or one V-cycle of the geometric
 * multigrid -- exactly the operator the Krylov solve applies (the PC setup of
 * the current T included).  Uses the solver's work vectors.  On a partition of
 * a box mesh (owned dofs in and out) the call is collective: every rank calls
 * it, through its communicator (the distributed or the per-slab V-cycle,
 * tv_options.mg_coupling). */
int tv_precond_apply(void* ctx, const double* r_dev, double* z_dev);

/* ---- solvers -------------------------------------------------------------- */
int tv_solve_T(void* ctx, int* newton_its, int* krylov_its, int* converged);
int tv_visco_update(void* ctx);
/* one time step (solve_timestep minus I/O); returns once the Newton solve has
 * converged, with the visco update still queued on the context's stream:
 * tv_get_field / tv_set_field / the operator calls / tv_field_device_ptr order
 * themselves behind it, tv_sync waits for it.  A Newton solve that reaches
 * newton_max_it unconverged returns TV_ERR_NOT_CONVERGED with the step's end
 * not run (dolfinx raises; T_prev and the visco state stay those of the
 * previous step), or -- error_on_nonconvergence = 0 -- ends the step anyway
 * (tv_last_converged tells; the reference's _solve_T would then fail its
 * assert(converged), ThermoViscoProblem.py:390) */
int tv_step(void* ctx, int thermal_only, int* newton_its, int* krylov_its);

/* ---- time-series output -------------------------------------------------------
 * The reference writes T, phi, Tf, xi (VTX/BP4) and sigma (XDMF/HDF5) every
 * step (ThermoViscoProblem.py:246-276 _write_initial_output, :357-364
 * _write_output, :614-620 _finalize).  Here: one XDMF 3 series per field
 * (<dir>/<name>.xdmf over raw little-endian <name>.bin, mesh_*.bin), written
 * asynchronously -- tv_output_write gathers the fields on the device, a copy
 * stream moves them to pinned host memory and a writer thread appends them to
 * the files while the next steps run; it blocks only when two writes are still
 * in flight.  tv_output_close drains.  A partition writes its owned nodes. */
int tv_output_open(void* ctx, const char* dir, const int* field_ids, int n_fields);
/* as tv_output_open, with the file stem of each series (<dir>/<name>.xdmf);
 * a NULL array or entry keeps the field's own name (setup()'s outfile_name /
 * outfile_name1, ThermoViscoProblem.py:176-178) */
int tv_output_open_named(void* ctx, const char* dir, const int* field_ids, const char* const* series_names,
                         int n_fields);
int tv_output_write(void* ctx, double t);
int tv_output_close(void* ctx);
/* The file format without a GPU (tests, tools): a rectilinear mesh as
 * tv_mesh_desc gives it (one partition), fields appended from host arrays in
 * the reference's interleaved layout; discontinuous = DG (cell-major dofs). */
void* tv_xdmf_open(const char* dir, int dim, const int* n_cells, const double* const* coords);
int tv_xdmf_add_field(void* xdmf, const char* name, int ncomp, int discontinuous);
int tv_xdmf_append(void* xdmf, int field, double t, const double* values, size_t n_values);
void tv_xdmf_close(void* xdmf);

/* ---- multi-GPU (one process per GPU, RCCL over xGMI) ---------------------- */
int tv_comm_unique_id_size(void);
int tv_comm_get_unique_id(char* id_out);   /* rank 0; broadcast it out-of-band */
int tv_comm_init(void* ctx, const char* id, int n_ranks, int rank);
int tv_halo_exchange(void* ctx, int field);
/* Host-staged communicator for running several partitions on one GPU (tests):
 * the library stages ghost planes / partial sums through pinned host memory
 * and calls these synchronously (return 0 on success).  Production multi-GPU
 * runs use tv_comm_init (RCCL). */
typedef int (*tv_host_allreduce_fn)(double* buf, int n, void* user);
typedef int (*tv_host_sendrecv_fn)(const double* send, size_t n_send, int peer_send, double* recv,
                                   size_t n_recv, int peer_recv, void* user);
/* Measurement only (bench.py --share): one rank's share of a partitioned run
 * on one GPU with the transport stubbed -- the multi-rank launch sequence,
 * every exchange fills the ghosts of the solver's vectors with zeros (the
 * partition solves its own block, so the operators stay SPD), the
 * temperature ghosts keep their values, every reduction stays local. */
int tv_comm_init_stub(void* ctx);   /* needs options.ksp_fixed_its > 0; tv_get_field and
                                       tv_output_write then refuse (TV_ERR_STATE) */
/* Transport test on ONE GPU: a one-rank RCCL communicator (id from
 * tv_comm_get_unique_id) on which every neighbour of this partition is the rank
 * itself -- the production RCCL groups run unchanged with self send/recv pairs
 * and one-rank all-reduces, so each ghost plane receives a boundary plane
 * this partition sends: a slab with neighbours on both sides sees its own
 * periodic images (ghost planes below <- its top owned planes, above <- its
 * bottom ones: one period of a periodic plate), a slab with one neighbour its
 * MIRROR image across the interface (ghost plane k_begin-1-j <- owned plane
 * k_begin+j, one send / receive pair per plane) -- either way the operator on
 * the owned planes stays symmetric.  tv_comm_init_host with n_ranks = 1 (rank 0)
 * on a partition is the same loopback over the host-staged transport, its
 * callback copying a send into its receive (tests/test_loopback.py compares
 * the two). */
int tv_comm_init_loopback(void* ctx, const char* id);
/* Collective check of the transport (every rank calls it): the exchange
 * patterns the solver issues -- ghost planes of the fine grid and of every
 * distributed multigrid level, the sums + ghosts group of a KSPCG iteration,
 * the single-reduction group, the replicated level's vector all-reduce, the
 * per-neighbour unstructured halo -- run on vectors of global node ids and are
 * compared on the host with what each ghost must receive.  n_bad = 0 when
 * every one of the n_checked received values is right.  Replaces nothing in
 * the reference (a pre-flight of :351's scatter_forward). */
int tv_comm_check(void* ctx, int64_t* n_checked, int64_t* n_bad);
int tv_comm_init_host(void* ctx, int n_ranks, int rank, tv_host_allreduce_fn allreduce_fn,
                      tv_host_sendrecv_fn sendrecv_fn, void* user);
/* Cost of one exchange pattern of the partitioned solve on the transport in
 * place (collective; measurement only -- it overwrites solver scratch): `reps`
 * back-to-back calls on the context stream between two HIP events, the mean
 * stream time per call in microseconds.  Patterns (TV_XCHG_*): the fine-grid
 * ghost planes, a one-scalar all-reduce, the closing group of a KSPCG
 * iteration (2 sums + the ghost planes of z), the replicated multigrid level's
 * vector all-reduce, the ghost planes of distributed multigrid level 1 / 2.
 * TV_ERR_ARG when the pattern does not occur on this context.  On a loopback
 * communicator (tv_comm_init_loopback) this is the fixed cost of each RCCL
 * group on one GPU -- a lower bound of the same group across xGMI. */
enum { TV_XCHG_HALO = 0, TV_XCHG_ALLREDUCE1 = 1, TV_XCHG_CLOSE = 2, TV_XCHG_VEC = 3, TV_XCHG_HALO_L1 = 4,
       TV_XCHG_HALO_L2 = 5, TV_XCHG_COUNT = 6 };
int tv_comm_time(void* ctx, int pattern, int reps, double* us_per_call);

/* ---- measurement ------------------------------------------------------------ */
/* time `reps` launches of one hot kernel on the context stream with HIP events;
 * kernel: 0 = Jacobian apply (matvec), 1 = fused viscoelastic update,
 * 2 = residual, 3 = fused PCG matvec (p <- z + b p; w <- J p; p.w),
 * 4 = PCG vector update, 10 = Jacobian apply with the 256 MiB Infinity Cache
 * flushed (512 MiB write) before every launch, events around the launch alone,
 * the MEDIAN over the reps, 11 = one GMG V-cycle.  Launch audit, 12-17: `reps`
 * back-to-back launches queued behind a spin kernel (timed as the GPU runs them,
 * not at the host's enqueue rate), events around the chain: 12 an empty
 * one-thread kernel, 13 the solver-state upload kernel, 14 the one-block
 * reduction, 15 a Jacobi sweep of the coarsest GMG level, 16 J x of GMG level 1,
 * 17 the fine J x.  Writes the duration per launch in ms (the mean, except 10). */
int tv_time_kernel(void* ctx, int kernel, int reps, double* ms_per_launch);
/* algorithmic bytes moved by one launch of `kernel` */
int tv_kernel_bytes(void* ctx, int kernel, double* bytes);
/* in-solve timing: with `on` > 0, every following tv_step times the fused PCG
 * matvec (kernel 3) and the PCG update (4) of every converging iteration
 * (on > 1: every on-th) from device clock stamps the launches write themselves
 * (first workgroup's start, reduction tail's end: what a kernel trace reports),
 * and the viscoelastic update (1) with HIP events; the counters restart at every
 * call.  Kernel 3 is timed on the 3D CG marching path only (launches 0 else).
 * tv_kernel_stats returns the mean duration (ms) and the number of timed launches. */
int tv_kernel_timing(void* ctx, int on);
int tv_kernel_stats(void* ctx, int kernel, double* ms_avg, int64_t* launches);
/* counters of the last tv_step / tv_solve_T */
int tv_last_stats(void* ctx, int* newton_its, int* krylov_its, double* dx_norm);
/* whether the last tv_step / tv_solve_T met the Newton test (with
 * error_on_nonconvergence = 0 an unconverged solve returns TV_OK) */
int tv_last_converged(void* ctx, int* converged);
/* the Krylov iteration form in use (TV_PCG_KSPCG or TV_PCG_SINGLE_REDUCTION:
 * the Jacobi march form, or with TV_PC_GMG the single-reduction GMG-PCG of
 * deep-ghost slabs, which only pcg_variant AUTO selects); with the Jacobi SINGLE_REDUCTION form, kernel id 3 of
 * tv_time_kernel / tv_kernel_bytes / tv_kernel_stats is the fused
 * single-reduction iteration and id 4 is unused (GMG: the ids keep their
 * meaning) */
int tv_pcg_variant(void* ctx, int* variant);

#ifdef __cplusplus
}
#endif
#endif /* TVFEM_H */
