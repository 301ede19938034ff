/*
 * pcd.h -- C-ABI of libpcd.so, the MI355X-native (gfx950) hot path of the normal-guided point-cloud denoiser.
 *
 * Every entry point takes raw DEVICE pointers + sizes + an opaque hipStream_t (passed as void*), never torch
 * types.  Calls are stream-ordered; the library never frees caller memory.  Every entry returns an int status
 * (PCD_OK = 0, negative on error) and pcd_last_error() returns a thread-local description of the last failure.
 * Numerical guards of the reference (Σw = 0 fallbacks, singular 3x3 masks, displacement clamps) are reproduced
 * and never raised.
 *
 * Reference interface each entry replaces (paths relative to the reference repository root):
 *   pcd_grid_build / pcd_grid_*    Selector.__init__ KDTree snapshot          Pointcloud/Modules/Selector.py:138-141
 *   pcd_knn                         Selector.getKNNSelection                   Pointcloud/Modules/Selector.py:235-246
 *                                   torch_cluster.knn_graph (loop=False)       Pointcloud/Modules/GraphBuilder.py:60-63
 *                                   torch_geometric.nn.pool.knn (k=1)          Pointcloud/Modules/Utils.py:253-295
 *   pcd_radius_count / _fill        Selector.getPointsInRangeSelection(Vectorized)  Pointcloud/Modules/Selector.py:214-233
 *   pcd_nvt_csr                     Decompositionor.getBetterFilteredNVT       Pointcloud/Modules/Decompositionor.py:278-300
 *   pcd_nvt_normal_csr              Decompositionor.getNormalFilteredNVT       Pointcloud/Modules/Decompositionor.py:260-276
 *   pcd_pvt_normal_csr              Decompositionor.getNormalFilteredPVT       Pointcloud/Modules/Decompositionor.py:172-211
 *   pcd_vu_smooth                   Decomposition.getVUSmoothedNormals         Pointcloud/Modules/Decompositionor.py:92-106
 *   pcd_classify                    Decomposition.getNVTFeatures/getClasses    Pointcloud/Modules/Decompositionor.py:57-69
 *   pcd_pca_dense                   GraphBuilder.getPVTDecompositionWithKNN    Pointcloud/Modules/GraphBuilder.py:99-111
 *   pcd_step_csr                    Denoiser.{flat,edge,feature,corner,new,dummy}_step  Pointcloud/Modules/Denoiser.py:26-232
 *   pcd_edge_length_sum             TorchUtils.averageEdgeLength               Pointcloud/Modules/Utils.py:297-299
 *   pcd_nn_dist                     TorchUtils.Chamfer/Paper/HausdorffDistance Pointcloud/Modules/Utils.py:253-295
 *   pcd_mesh_update(_f32)           Mesh.updateVertices                        PatchGeneration/Modules/Mesh.py:377-418
 *   pcd_mesh_vta                    igl.vertex_triangle_adjacency (Mesh.__init__) PatchGeneration/Modules/Mesh.py:26
 *   pcd_denoiser_*                  Processor.denoise / getMyFeatureDecomposition / denoiseUntilMinimumError loop body
 *                                                                              Pointcloud/Modules/Processor.py:110-185
 *   pcd_orient_normals_mst          GraphBuilder.flipNormals (MST + DFS, host) Pointcloud/Modules/GraphBuilder.py:129-209
 *   pcd_orient_normals_mst_gpu      GraphBuilder.flipNormals (Borůvka MST + Euler-tour rooting + sign pointer jumping,
 *                                   device)                                    Pointcloud/Modules/GraphBuilder.py:129-209
 */
#ifndef PCD_H
#define PCD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ status */
enum {
    PCD_OK = 0,
    PCD_ERR_ARG = -1,      /* bad argument (null pointer, size, unsupported k)     -> AssertionError/ValueError */
    PCD_ERR_OOM = -2,      /* device allocation failed                               */
    PCD_ERR_HIP = -3,      /* HIP runtime error                                      */
    PCD_ERR_STATE = -4,    /* object used in the wrong state                          */
    PCD_ERR_RCCL = -5      /* collective failure (multi-GPU slab mode)                */
};
const char* pcd_last_error(void);
int pcd_version(void);
/* hash of the sources and flags this library was built from (16 hex digits), e.g. to match profiles to builds */
const char* pcd_build_id(void);
/* Largest k supported by the kNN kernels (register top-k lists). */
int pcd_max_k(void);

/* ------------------------------------------------------------------ frozen snapshot (H1) */
typedef struct pcd_grid pcd_grid;
typedef struct {
    int64_t n;           /* snapshot points                           */
    int64_t cells;       /* occupied cells                            */
    int64_t table_slots; /* hash-table slots                          */
    float cell;          /* cell edge length                          */
    float origin[3];     /* cell (0,0,0) lower corner                  */
    int32_t dims[3];     /* cells per axis over the snapshot bbox       */
} pcd_grid_info_t;

/* Build the kNN index over a private copy of xyz[n][3] (fp32 device rows).  cell <= 0 picks the cell edge
 * so an occupied cell holds ~k_hint/2 points.  origin3 (host, nullable; needs cell > 0) pins the cell lattice:
 * grids of subsets built on one lattice order their points as subsequences of the full set's order (used by
 * the spatial slabs, so every rank breaks distance ties like one GPU would).  Synchronises `stream`.
 * Replaces the KDTree construction of Selector.__init__ (Pointcloud/Modules/Selector.py:138-141). */
int pcd_grid_build(const float* xyz, int64_t n, int k_hint, float cell, const float* origin3, void* stream,
                   pcd_grid** out);
/* The cell lattice pcd_grid_build would pick for xyz (origin = bbox minimum, cell edge), without building. */
int pcd_grid_params(const float* xyz, int64_t n, int k_hint, float cell, float* origin3, float* cell_out,
                    void* stream);
/* Another index over the SAME frozen snapshot as `src` (its points, in caller order) with another cell size (cell <= 0:
 * ~k_hint/2 points per occupied cell).  The fused loop indexes its snapshot with cells of about its list cap
 * (Processor picks k_hint = 2 x the cap): the re-anchoring searches then resolve fewer, fuller cells per query.
 * Synchronises `stream`. */
int pcd_grid_rebuild(const pcd_grid* src, int k_hint, float cell, void* stream, pcd_grid** out);
int pcd_grid_destroy(pcd_grid* g);
int pcd_grid_get_info(const pcd_grid* g, pcd_grid_info_t* out);
/* perm[r] = original index of the r-th point in the grid's spatial (Morton) order; int32 device [n]. */
int pcd_grid_perm(const pcd_grid* g, int32_t* perm, void* stream);

/* ------------------------------------------------------------------ kNN (H2) */
/* For each query row q[nq][3] the k nearest snapshot points, ascending (d², index).
 *   idx_bits    32 or 64: element type of idx_out ([nq][k] row-major)
 *   sorted_ids  0: indices in the caller's original order, 1: indices in the grid's spatial order
 *   exclude_self  1: query i is snapshot point i; drop it (torch_cluster.knn_graph loop=False semantics)
 *   d2_out      nullable fp32 [nq][k] squared distances */
int pcd_knn(const pcd_grid* g, const float* q, int64_t nq, int k, void* idx_out, int idx_bits, int sorted_ids,
            int exclude_self, float* d2_out, void* stream);

/* Radius selection over the frozen snapshot (scipy query_ball_point semantics: float64 ((dx²+dy²)+dz²) <= r²,
 * members in ascending ORIGINAL index).  Two calls: count [nq] (int64), then, with the caller's exclusive prefix
 * sums offsets [nq+1] and total = offsets[nq], fill idx_out [total] (int64).  fill synchronises `stream`.
 * radii: fp32 [nq] per query (the reference builds a torch.float radius tensor, Selector.py:233). */
int pcd_radius_count(const pcd_grid* g, const float* q, int64_t nq, const float* radii, int64_t* counts,
                     void* stream);
int pcd_radius_fill(const pcd_grid* g, const float* q, int64_t nq, const float* radii, const int64_t* offsets,
                    int64_t total, int64_t* idx_out, void* stream);

/* Diagnostic: total work of a kNN(k) pass over q (spatial-order ids), summed over queries into out6 (device u64):
 * cells considered, cells probed in the hash, cells found, candidates scanned, sorted inserts (variant 0:
 * per-candidate insertion) or batch merges (variant 1: batched search, k > 8), extra rings. */
int pcd_knn_stats(const pcd_grid* g, const float* q, int64_t nq, int k, int variant, unsigned long long* out6,
                  void* stream);

/* ------------------------------------------------------------------ tensor voting (H5-H7, H15) */
/* CSR selection: segment r has centre ci[r] and neighbours nbr[off[r] .. off[r+1]); all int64 (torch long). */
int pcd_nvt_csr(const float* pos, const float* n, int64_t npts, const int64_t* ci, const int64_t* off,
                const int64_t* nbr, int64_t m, float rho, float* eigval, float* eigvec, void* stream);
/* Normal-filtered NVT (CPSD): w_ij = acos(clamp(n_i . n_j)) <= rho; T_i = sum w n_j n_j^T / sum w, or n_i n_i^T when
 * no neighbour votes.  Same CSR and outputs as pcd_nvt_csr. */
int pcd_nvt_normal_csr(const float* n, int64_t npts, const int64_t* ci, const int64_t* off, const int64_t* nbr,
                       int64_t m, float rho, float* eigval, float* eigvec, void* stream);
/* Normal-filtered PVT (CPSD): same vote; every w := 1 when none votes; weighted covariance of v_j about their
 * weighted mean / sum w; an empty neighbourhood gets the reference's cross-product samples.  Outputs as above. */
int pcd_pvt_normal_csr(const float* pos, const float* n, int64_t npts, const int64_t* ci, const int64_t* off,
                       const int64_t* nbr, int64_t m, float rho, float* eigval, float* eigvec, void* stream);
/* eigval [m][3] ascending, eigvec [m][3][3] (columns), n [m][3] -> f_n [m][3] */
int pcd_vu_smooth(const float* eigval, const float* eigvec, const float* n, int64_t m, float tau, float damp,
                  float* out, void* stream);
/* features nullable [m][3] = (planarity, linearity, sphericity); classes int64 [m] */
int pcd_classify(const float* eigval, int64_t m, float scale, float* features, int64_t* classes, void* stream);
/* The kernels' two 3x3 symmetric eigen-solvers on DEVICE tensors t6 [m][6] = (a00, a01, a02, a11, a12, a22), as
 * the fused loop compiles them (torch.linalg.eigh at Decompositionor.py:300 is what both replace):
 *   solver 0: the LAPACK ssyevd restatement (NVT1, the public ops) -> w [m][3] ascending, vec [m][3][3] columns
 *   solver 1: NVT2's fixed-sweep Jacobi on the hardware rcp/sqrt estimates -> w [m][3] ascending, vec [m][3] = the
 *             smallest eigenvalue's unit eigenvector (sign arbitrary; classes and edge_step use it through y yᵀ)
 * For tests: pins NVT2's solver against the LAPACK one on the same tensors. */
int pcd_eigh3_batch(const float* t6, int64_t m, int solver, float* w, float* vec, void* stream);
/* Covariance of the k neighbours nbr[i*k .. i*k+k) about their own mean; eigval [n][3], eigvec [n][3][3]. */
int pcd_pca_dense(const float* pos, int64_t n, const int64_t* nbr, int k, float* eigval, float* eigvec,
                  void* stream);

/* ------------------------------------------------------------------ position updates (H9-H12) */
enum { PCD_STEP_FLAT = 0, PCD_STEP_EDGE = 1, PCD_STEP_FEATURE = 2, PCD_STEP_CORNER = 3, PCD_STEP_NEW = 4,
       PCD_STEP_DUMMY = 5 };
/* One Denoiser.*_step over a CSR selection: out [m][3] new positions of the centres.
 * edge_vectors [npts][3] is required for PCD_STEP_EDGE only.  Uses a device workspace it allocates
 * internally for the global (flat/new) reductions; stream-ordered. */
int pcd_step_csr(int kind, const float* pos, const float* n, const float* edge_vectors, int64_t npts,
                 const int64_t* ci, const int64_t* off, const int64_t* nbr, int64_t m, float d, float alpha,
                 float* out, void* stream);

/* ------------------------------------------------------------------ metrics (H4, H17) */
/* sum over rows of ||pos[b[e]] - pos[a[e]]|| in fp64 -> *sum_out (device double) */
int pcd_edge_length_sum(const float* pos, const int64_t* a, const int64_t* b, int64_t e, double* sum_out,
                        void* stream);
/* for each query: squared distance to / index of its nearest snapshot point (k = 1) */
int pcd_nn_dist(const pcd_grid* g, const float* q, int64_t nq, float* d2_out, int64_t* idx_out, void* stream);

/* ------------------------------------------------------------------ mesh vertex update (H18) */
/* k Jacobi sweeps of v_i += Σ_{f∋i} Σ_{c∈f} n_f (n_f·(v_c − v_i)) / (3 deg_i), fp64, in place on v [nv][3].
 * f [nf][3] int64, fn [nf][3] f64, vf/ni = igl vertex_triangle_adjacency (VF [3nf], NI [nv+1]) int64. */
int pcd_mesh_update(double* v, int64_t nv, const int64_t* f, const double* fn, int64_t nf, const int64_t* vf,
                    const int64_t* ni, int k, void* stream);
/* The same k Jacobi sweeps in fp32 (v [nv][3] f32 in place, f [nf][3] int32, fn [nf][3] f32, vf / ni int32): vertex and
 * normal rows as float4 and faces as int4 internally, one thread per vertex.  Not bitwise the fp64 path: within fp32
 * rounding of it (tests/test_gpu_mesh.py). */
int pcd_mesh_update_f32(float* v, int64_t nv, const int32_t* f, const float* fn, int64_t nf, const int32_t* vf,
                        const int32_t* ni, int k, void* stream);
/* igl.vertex_triangle_adjacency (the reference's Mesh.__init__, PatchGeneration/Modules/Mesh.py:26) on the device:
 * f [nf][3] (int32 or int64 per f_bits) -> vf [3 nf] (the incident faces of each vertex in increasing face order) and
 * ni [nv + 1] offsets, int32 or int64 per out_bits.  PCD_ERR_ARG for a face index outside [0, nv).  Synchronises. */
int pcd_mesh_vta(const void* f, int f_bits, int64_t nf, int64_t nv, void* vf, void* ni, int out_bits, void* stream);

/* ------------------------------------------------------------------ fused denoise loop (H8, H13, H14) */
typedef struct pcd_denoiser pcd_denoiser;
typedef struct {
    int k;               /* feature kNN size (getMyFeatureDecomposition N), reference default 16       */
    int k_update;        /* update kNN size, reference 8                                                 */
    float rho;           /* NVT angle threshold, reference 5*pi/12                                       */
    float tau;           /* VU smoothing eigenvalue threshold, reference 0.3                             */
    float damp;          /* VU smoothing dampening d, reference 3                                        */
    float class_scale;   /* planarity scale in getClasses, reference 0.2                                 */
    float d;             /* displacement clamp (2 * mean edge length in Processor.denoise)              */
    int nphases;         /* number of (class, step, alpha) phases, Gauss-Seidel in this order           */
    int phase_class[3];  /* 0 flat, 1 edge, 2 corner                                                     */
    int phase_kind[3];   /* PCD_STEP_*                                                                   */
    float phase_alpha[3];
    int jacobi;          /* 0: Gauss-Seidel across the phases (Processor.denoise, Processor.py:127-138); 1: every phase
                            reads the iteration's input positions (Jacobi across classes: temp_pos, the thesis driver
                            "Ours", PostProcessing.ipynb:1069-1090)                                          */
    float clamp_global;  /* > 0: a moved point keeps its new position only while it lies within clamp_global of its
                            position at pcd_denoiser_load, else it keeps the previous iteration's position
                            (PostProcessing.ipynb:1088-1089, mask = ||temp_pos - original_pos|| < d); 0: off */
} pcd_denoise_params;

/* sizeof(pcd_denoise_params) as this library was built: a binding checks its mirror against it (a struct that
 * is shorter than the library's would be read past its end). */
int pcd_denoise_params_size(void);
/* g: the frozen snapshot, fewer than 2^27 points (134M; larger clouds run as spatial slabs, pcd_slab). */
int pcd_denoiser_create(const pcd_grid* g, int k_max, pcd_denoiser** out);
int pcd_denoiser_destroy(pcd_denoiser* dn);
/* pos, n: caller rows [N][3] (original order, N = grid n) -> internal spatial order */
int pcd_denoiser_load(pcd_denoiser* dn, const float* pos, const float* n, void* stream);
int pcd_denoiser_iterate(pcd_denoiser* dn, const pcd_denoise_params* p, int iterations, void* stream);
/* back to original order; any output pointer may be null.  classes int64 [N] and edge vectors [N][3]
 * are those of the LAST iteration's NVT2; f_n is the last smoothed normal field (= n after iterate). */
int pcd_denoiser_store(pcd_denoiser* dn, float* pos, float* n, int64_t* classes, float* edge_vectors,
                       void* stream);
/* Seeded search (default ON): iterations after the first cap the acceptance threshold at the largest key of
 * the previous iteration's stored list (re-keyed at the current positions) and run the capped search (LDS row
 * buffer, one sorted drain).  Results are identical either way (tested bitwise); it only changes the work done.
 * reset_seed forgets the stored list, so the next iterate() runs unseeded. */
int pcd_denoiser_set_seeding(pcd_denoiser* dn, int enable);
/* LDS row windows (default ON): NVT1, NVT2 and the flat phase stage a window of rows around each block's own rows
 * in LDS and read neighbours from it when they fall inside.  OFF reads every neighbour from global memory: same
 * results bit for bit (the parity tests check this); a diagnostic / reference switch. */
int pcd_denoiser_set_windows(pcd_denoiser* dn, int enable);
int pcd_denoiser_reset_seed(pcd_denoiser* dn);
/* Anchored search (default ON, applies to seeded searches with k, k_update <= 32): each point keeps an anchor --
 * a position, the exact 2K nearest snapshot points there (K = the list cap 8/16/32) and their 2K-th distance D.
 * When the current k-th distance over that list is below D - |q - anchor|, the list's top k IS the snapshot's
 * k-NN (no grid search); the few queries that fail are re-anchored by a wave-per-query grid search (the rare
 * query whose quantised ordering is ambiguous by the exact-key search).  Same results (tested bitwise).  Anchors depend only on the snapshot: they survive load(); reset_seed drops them. */
int pcd_denoiser_set_anchoring(pcd_denoiser* dn, int enable);
/* Diagnostics: rows re-anchored by the last anchored kNN stage (-1: none ran).  Synchronises `stream`. */
int pcd_denoiser_anchor_stats(pcd_denoiser* dn, int64_t* redo_rows, void* stream);
/* Diagnostics of the last anchored kNN stage: out4 = {rows re-anchored, of which spilled from the quantised-key
 * search to the exact-key wave search, of those: with a cap box over 4096 cells, with an ambiguous quantised order
 * or too few points under a dense cap}; -1 when no anchored stage ran.  Synchronises `stream`. */
int pcd_denoiser_tile_stats(pcd_denoiser* dn, int64_t* out4, void* stream);
/* Profiling aid: with timing enabled, every iteration (up to 256) records HIP events on its stream between the
 * stages; get_timing returns each stage's elapsed ms AVERAGED over the iterations recorded since set_timing or
 * the previous get_timing, then starts over.  Slots: anchor test (+ redo-list select), re-anchoring search, exact-key
 * spill search, NVT1 (the four make up K1: kNN + NVT1; a non-anchored K1 reports its whole time in the NVT1 slot),
 * NVT2, phase 0, phase 1, phase 2, finish, -.  enable = 2 records the K1 stage's two events only (one slot: K1's
 * ms), for a timed region that needs K1's time without the other stages' events (~4 us each on the stream). */
int pcd_denoiser_set_timing(pcd_denoiser* dn, int enable);
int pcd_denoiser_get_timing(pcd_denoiser* dn, float* ms_out, int n_slots, int* n_written);
/* Device error word -> status: PCD_ERR_STATE if a kNN list held an invalid entry or (spatial slabs) a query's
 * k-ball left the coverage box.  Synchronises `stream`.  store() calls it. */
int pcd_denoiser_check(pcd_denoiser* dn, void* stream);
/* The raw device error word behind check (bit 0: invalid list entry, bit 1: a k-ball left the coverage box; with bit
 * 1, bit 2: a row without a coverage sphere failed -- the band -- and bit 3: a sphere row failed), without raising:
 * the spatial-slab driver re-plans on bit 1.  Synchronises `stream`. */
int pcd_denoiser_status(pcd_denoiser* dn, int* bits, void* stream);
/* What the failed coverage checks lacked, for a re-plan that grows only that (spatial slabs; no reference
 * counterpart): band_excess = the farthest any sphere-less row's k-ball reached past the coverage box
 * (0: none failed), sphere_ratio = the largest (|q - centre| + d_k) / R over the sphere rows that failed (0: none).
 * Synchronises `stream`. */
int pcd_denoiser_coverage_excess(pcd_denoiser* dn, float* band_excess, float* sphere_ratio, void* stream);
/* The kNN list the last K1 stage stored (the snapshot's `cols` nearest of each point's current position, in
 * (distance, index) order = getKNNSelection's columns, Selector.py:235-246), in caller order with ORIGINAL snapshot
 * indices: out int64 [N][cols], cols <= the stored list length (max(k, k_update) of the last iteration). */
int pcd_denoiser_lists(pcd_denoiser* dn, int64_t* out, int cols, void* stream);
/* Parity probe of the fused NVT2 stage (off by default; enabling allocates [N] float4).  While on, every NVT2 stage
 * also writes, per row, the eigenvalues of the reference's normalised tensor T / Σw (Decompositionor.py:299-300:
 * getBetterFilteredNVT's eigval, ascending) and Σw, as that kernel computes them.  probe_store copies them out in
 * caller order: nvt2_eig4 [N][4] = (λ0, λ1, λ2, Σw); rows no NVT2 stage wrote hold NaN.  The edge vectors (the
 * smallest eigenvalue's eigenvector) come out through pcd_denoiser_store. */
int pcd_denoiser_set_probe(pcd_denoiser* dn, int enable);
int pcd_denoiser_probe_store(pcd_denoiser* dn, float* nvt2_eig4, void* stream);

/* ---- spatial slabs (multi-GPU): the same loop over a rank's own points with a halo ----
 * The grid holds the rank's points plus halo snapshot points owned by other ranks.  Only the ACTIVE rows are
 * queried and updated; the caller keeps the halo rows' state current with pack/unpack + its own transport
 * (RCCL) between stages, and all-reduces the flat-phase sums (sum) and delta (max) between the PHASE_* stages:
 *   per iteration: KNN_NVT1 -> exchange FN -> NVT2 -> per phase [flat/new: PHASE_SUM(red=double[4]) ->
 *   all-reduce sum -> PHASE_CENTRE(red) -> PHASE_MAXDIST(red=float[1]) -> all-reduce max] -> PHASE_APPLY(red or
 *   null) -> exchange POS -> FINISH.  pcd_denoiser_iterate runs the same sequence with no exchange. */
enum { PCD_FIELD_POS = 0, PCD_FIELD_NRM = 1, PCD_FIELD_FN = 2, PCD_FIELD_EDGE = 3 };
enum { PCD_STAGE_KNN_NVT1 = 0, PCD_STAGE_NVT2 = 1, PCD_STAGE_PHASE_SUM = 2, PCD_STAGE_PHASE_CENTRE = 3,
       PCD_STAGE_PHASE_MAXDIST = 4, PCD_STAGE_PHASE_APPLY = 5, PCD_STAGE_FINISH = 6 };
/* rows: device int32 [n_rows] of spatial-order rows (ascending), kept by the caller; null = all rows. */
int pcd_denoiser_set_rows(pcd_denoiser* dn, const int32_t* rows, int64_t n_rows);
/* host lo3/hi3: the box the local snapshot covers (null: no check). */
int pcd_denoiser_set_coverage(pcd_denoiser* dn, const float* lo3, const float* hi3);
/* Spatial slabs: per-point coverage spheres (DEVICE float [n], caller order; 0 = none; null: clear).  A point whose
 * k-ball leaves the coverage box is still covered when the ball lies inside the sphere of radius radii[i] around its
 * position at load -- the slab driver adds every snapshot point of such a sphere to the local snapshot (the sparse
 * points near a cut, whose balls would otherwise widen every rank's halo).  Replaces nothing in the reference (it is
 * the exactness condition of Selector.getKNNSelection's KD-tree query over a partitioned snapshot, Selector.py:243). */
int pcd_denoiser_set_coverage_spheres(pcd_denoiser* dn, const float* radii, void* stream);
/* one stage; red: device scalars as above (SUM/CENTRE: double[4] Σx,Σy,Σz,count; MAXDIST out / APPLY in:
 * float[1] delta, nullable = local value). */
int pcd_denoiser_stage(pcd_denoiser* dn, const pcd_denoise_params* p, int stage, int phase, void* red,
                       void* stream);
/* state rows <-> packed device float4 buffers (field PCD_FIELD_*; POS = current positions, EDGE = NVT2's edge vectors,
 * written by a test to feed the edge phase the reference's own).  FN rows unpacked
 * between K1 and NVT2 must be another rank's K1 output (unit vectors: NVT2's vote margin assumes it). */
int pcd_denoiser_pack(pcd_denoiser* dn, int field, const int32_t* rows, int64_t n, float* out4, void* stream);
int pcd_denoiser_unpack(pcd_denoiser* dn, int field, const int32_t* rows, int64_t n, const float* in4,
                        void* stream);

/* ---- the CPSD ("Martin") comparison driver in one call (PostProcessing.ipynb:1041-1062) ----
 * Per iteration on the loaded state: kNN(k_update) lists of the current positions, the radius-r selection over the
 * frozen snapshot (scipy query_ball_point membership, Selector.py:214-233) with the normal-filtered NVT + VU smoothing
 * (Processor.getMartinFeatureDecomposition, Processor.py:102-108) and PVT, VU features (Decompositionor.py:84-85), then
 * flat_step / edge_step / corner_step with alpha[3] and the per-step clamp, Jacobi across classes, the global clamp
 * ||pos - pos at load|| < d, n := f_n.  No host synchronisation per iteration; one at the end of the call. */
typedef struct {
    float r;             /* radius of the selection, the notebook's r = d                               */
    float rho;           /* vote angle of both normal filters, 0.9                                      */
    float tau;           /* VU smoothing and VU-feature threshold, 0.3                                  */
    float damp;          /* VU smoothing dampening, 3                                                   */
    float d;             /* global clamp (PostProcessing.ipynb:1060)                                    */
    float step_clamp;    /* per-step displacement clamp, d * 20000                                      */
    float alpha[3];      /* flat, edge, corner step: 0.1, 1, 1                                          */
    int k_update;        /* update kNN size, 8                                                          */
} pcd_cpsd_params;
int pcd_cpsd_iterate(pcd_denoiser* dn, const pcd_cpsd_params* p, int iterations, void* stream);

/* ---- spatial slabs in one call per iteration (the RCCL communicator, halo exchange and scalar
 * all-reduces live in the library; PyTorch only sets up the ranks) ----
 * A pcd_comm is the slab transport: RCCL over xGMI (pcd_comm_create from a unique id rank 0 made with pcd_comm_id and
 * the caller broadcast), or host callbacks (pcd_comm_create_host: any transport the caller has, e.g. gloo in tests;
 * every exchange is staged through pinned host memory and handed to the callback). */
typedef struct pcd_comm pcd_comm;
enum { PCD_DT_F32 = 0, PCD_DT_F64 = 1, PCD_DT_I32 = 2 };
enum { PCD_OP_SUM = 0, PCD_OP_MAX = 1 };
typedef struct {
    void* user;
    /* Exchange float4 rows with npeers peers: to peers[q] send rows [send_off[q], send_off[q+1]) of `send`, from it
     * receive rows [recv_off[q], recv_off[q+1]) into `recv` (HOST memory, 4 floats a row).  Return 0 on success. */
    int (*exchange)(void* user, int npeers, const int* peers, const float* send, const int64_t* send_off, float* recv,
                    const int64_t* recv_off);
    /* In-place all-reduce of count elements of dtype PCD_DT_* with PCD_OP_* over every rank (HOST memory). */
    int (*allreduce)(void* user, void* buf, int count, int dtype, int op);
} pcd_host_transport;
/* bytes of an RCCL unique id (ncclUniqueId) */
int pcd_comm_id_bytes(void);
/* rank 0: a fresh RCCL unique id into id_out [pcd_comm_id_bytes()] for the caller to broadcast */
int pcd_comm_id(void* id_out);
/* every rank (collective, on its own HIP device): the RCCL communicator of `world` ranks from rank 0's id */
int pcd_comm_create(const void* id, int world, int rank, pcd_comm** out);
int pcd_comm_create_host(const pcd_host_transport* t, int world, int rank, pcd_comm** out);
int pcd_comm_destroy(pcd_comm* c);
/* world size, this rank, and the transport (PCD_COMM_RCCL / PCD_COMM_HOST) the communicator was made with */
enum { PCD_COMM_HOST = 0, PCD_COMM_RCCL = 1 };
int pcd_comm_info(const pcd_comm* c, int* world, int* rank, int* transport);
/* Point-to-point bulk copy of DEVICE memory, stream-ordered: send send_bytes from `send` to rank send_peer and
 * receive recv_bytes into `recv` from rank recv_peer (a peer of -1: nothing that way).  Byte counts are multiples of
 * 4.  The slab driver's coordinator (rank 0, the only rank holding the whole cloud, as the reference's single process
 * does: Processor.py:115-121) hands each rank its slab + halo of the snapshot with it, and collects the owned state
 * for a re-plan.  RCCL: ncclSend / ncclRecv in one group.  Host transport: staged through host memory and handed to
 * the exchange callback as ceil(bytes / 16) float4 rows.  Synchronises `stream` on the host transport only. */
int pcd_comm_sendrecv(pcd_comm* c, int send_peer, const void* send, int64_t send_bytes, int recv_peer, void* recv,
                      int64_t recv_bytes, void* stream);
/* in-place all-reduce of device scalars (the flat phase's Σ and δ, Denoiser.py:106-107), stream-ordered */
int pcd_allreduce_scalars(pcd_comm* c, void* buf, int count, int dtype, int op, void* stream);
/* Halo routes of this rank's denoiser: for each of npeers peers (host arrays), n_send[q] own rows to send and
 * n_recv[q] halo rows to receive; send_rows / recv_rows: device int32 spatial-order rows, peer after peer (copied).
 * own_lo3 / own_hi3 (host, nullable): the OWNED slab (no halo) -- with it, NVT2 and the phases run the rows whose
 * k-ball stays strictly inside it while an exchange is in flight.  Synchronises `stream`. */
int pcd_denoiser_set_routes(pcd_denoiser* dn, int npeers, const int* peers, const int64_t* n_send,
                            const int32_t* send_rows, const int64_t* n_recv, const int32_t* recv_rows,
                            const float* own_lo3, const float* own_hi3, void* stream);
/* one field (PCD_FIELD_*) of the send rows -> the peers' halo rows, stream-ordered */
int pcd_halo_exchange(pcd_denoiser* dn, pcd_comm* c, int field, void* stream);
/* `iterations` slab iterations of Processor.denoise's body (Processor.py:123-139) over the active rows: K1, f_n
 * exchange, NVT2, the phases with their all-reduces and position exchanges, n := f_n -- one call, every exchange
 * overlapped with the rows that need no halo data (the exchange runs on a stream of the library's own; later
 * calls on this denoiser wait for it).  Same result bit for bit as the staged sequence above. */
int pcd_slab_iterate(pcd_denoiser* dn, pcd_comm* c, const pcd_denoise_params* p, int iterations, void* stream);
/* Read-set exchange (on by default; PCD_SLAB_READSET=0 in the environment at pcd_denoiser_set_routes, or on = 0
 * here: every halo row in every exchange).  pcd_slab_iterate's K1 stores the kNN lists first; each rank marks the
 * halo rows the lists of its band rows (k-ball not inside the owned slab) hold, sends that mask to each peer (one bit
 * per route row), and the peers send position + normal of exactly those rows while NVT1 runs the no-halo rows; the
 * iteration's f_n and position exchanges move the same rows, and no exchange trails the iteration.  The halo rows a
 * list does not hold are not kept current (pcd_halo_exchange refreshes every one).  Needs the anchored K1 (list cap
 * <= 32, seeding and anchoring on) and >= 2k local rows on every rank. */
int pcd_denoiser_set_readset(pcd_denoiser* dn, int on);
/* since pcd_denoiser_set_routes: read-set iterations and the send / receive rows they moved, summed */
int pcd_denoiser_readset_stats(const pcd_denoiser* dn, int64_t* iterations, int64_t* send_rows, int64_t* recv_rows);

/* ------------------------------------------------------------------ normal orientation (host) */
/* GraphBuilder.flipNormals: Kruskal MST on cost 1-|n_i·n_j| over the directed edge list (a[e] -> b[e],
 * host int64 arrays), then DFS from argmax z flipping n_dst when n_src·n_dst < cos(7π/12).  HOST memory,
 * n [npts][3] fp32 modified in place. */
int pcd_orient_normals_mst(const float* pos, float* n, int64_t npts, const int64_t* a, const int64_t* b,
                           int64_t e);
/* Same contract and bit-identical result on DEVICE memory (pos [npts][3], n [npts][3] in place, a/b [e] int64),
 * ordered on `stream`; synchronises the stream before returning.  The minimum spanning forest is unique under
 * keys (cost, edge index), which is the host's stable Kruskal order, and each node's sign is a composition of
 * per-edge maps {identity, negate, +1} from the root's sign, so the DFS visit order never matters.
 * PCD_ERR_ARG for an out-of-range edge index; npts and e must be < 2^32. */
int pcd_orient_normals_mst_gpu(const float* pos, float* n, int64_t npts, const int64_t* a, const int64_t* b,
                               int64_t e, void* stream);

/* ------------------------------------------------------------------ host builds of the per-point math */
/* The exact __host__ __device__ code the kernels run, compiled for the CPU (HOST pointers); for tests.
 *   t6 [m][6] = (a00, a01, a02, a11, a12, a22) -> w [m][3] ascending, v [m][3][3] columns (LAPACK ssyevd signs) */
int pcd_host_eigh3(const float* t6, int64_t m, float* w, float* v);
int pcd_host_vu_smooth(const float* w, const float* v, const float* n, int64_t m, float tau, float damp, float* out);
/* getBetterFilteredNVT's tensor T (before eigh) for CSR rows: centres ci [m], neighbours nbr[off[r] .. off[r+1]),
 * pos / n [.][3] -> t6 [m][6] (a00, a01, a02, a11, a12, a22); the fused kernels' vote and sums, on the host. */
int pcd_host_nvt_tensor(const float* pos, const float* n, const int64_t* ci, const int64_t* off, const int64_t* nbr,
                        int64_t m, float rho, float* t6);
/* a9 [m][3][3] row-major, b3 [m][3] -> x3 [m][3] = inv_ex(A) b as the position steps compute it, ok [m] (0 when
 * inv_ex reports info != 0, i.e. an exactly zero pivot; x untouched = 0) */
int pcd_host_solve3(const float* a9, const float* b3, int64_t m, float* x3, int32_t* ok);
/* torch.linalg.inv_ex (Denoiser.py:43, 80, 163, 210) restated for 3x3: a9 [m][3][3] -> inv9 [m][3][3], ok [m] as
 * above (inv untouched = 0 where ok = 0).  The position steps' arithmetic (pcd_device.h inv3_ref), on the host. */
int pcd_host_inv3(const float* a9, int64_t m, float* inv9, int32_t* ok);
/* Denoiser.*_step (PCD_STEP_*) over CSR rows, the kernels' step functions on the host: out [m][3]; delta = the global
 * flat / new-step delta (Denoiser.py:107, 138). */
int pcd_host_step_csr(int kind, const float* pos, const float* n, const float* edge_vectors, const int64_t* ci,
                      const int64_t* off, const int64_t* nbr, int64_t m, float delta, float d, float alpha, float* out);

#ifdef __cplusplus
}
#endif
#endif /* PCD_H */
