/* shud_partition.h — C-ABI of the C++ mesh partitioner and halo planner (libshud_host.so, plain C++).
 *
 * the reference runs its RHS as one OpenMP loop over all elements (src/ModelData/MD_f_omp.cpp:
 * 12-66, MD_f.cpp:9-50); here the mesh is split across one process per GPU, each rank computes the fluxes
 * of the elements and reaches it owns, and one halo exchange per RHS ships the ghost states.  METIS is not
 * in the image, so the partitioner is our own multilevel scheme (SHUD_PART_MULTILEVEL):
 *   graph      element dual graph: one edge per shared mesh edge (weight 1) plus river coupling (weight 1
 *              each): consecutive segments of a reach (.sp.rivseg order) and a reach's last segment to its
 *              downstream reach's first; vertex weight 1 + #segments of the element
 *   coarsening heavy-edge matching in seeded random order, contraction until ~200 vertices are left,
 *              once per bisection of a recursive bisection
 *   initial    greedy graph growing from 12 seeds on the coarsest graph, each refined by Fiduccia–Mattheyses
 *              passes (max-gain heap, hill climbing with rollback to the best cut); the best is kept
 *   refinement FM passes at every uncoarsening level of each bisection (the per-bisection balance slack
 *              is 1.03^(1/log2 k) so the k-way result stays within a 1.03 weight cap), then one k-way greedy
 *              boundary pass over the assembled partition (positive-gain and balance-improving moves)
 * SHUD_PART_RCB is the weighted recursive coordinate bisection fallback (the Python tests' partitioner,
 * bit-identical: shud-up_amd/shud_rhs/partition.py rcb).  SHUD_PART_AUTO runs both and keeps the partition
 * whose largest per-rank halo (ghost elements + ghost reaches) is smaller: on the reference's irregular basin
 * meshes the multilevel partition wins; on the jittered-grid synthetic mesh straight RCB cuts can.
 *
 * Ownership and halo plans follow partition.py: reach -> part owning most of its segments' elements (ties:
 * lowest part; no segments: part 0); a segment belongs to every rank owning its element or its reach.  Local
 * numbering of rank r: elements [owned interior | owned boundary | ghosts grouped by source rank], reaches
 * [owned | ghosts grouped by source rank], each group in global order; boundary = owned elements that read
 * ghost data.  The plan fills ShudPartition (include/shud_rhs.h) and the local ShudMeshSoA / ShudParamsSoA
 * for shud_rhs_create_partitioned; owned results are then bit-identical to one GPU.
 *
 * Lakes (serial semantics): a lake's sums (its elements' PET / precipitation, its bank edges'
 * fluxes, its inflowing reaches' QrivDown — MD_f.cpp:12-17,180-191) must be formed on one rank, so a lake
 * group — the elements of a lake, the non-lake elements with an edge on it (bank elements), and lakes that
 * touch through a shared bank element or adjacent lake elements — always lies on one part: shud_partition_mesh
 * moves each group to the part already holding most of its weight (shud_partition_constrain does the same for
 * a caller's partition), and a reach with a segment on a lake element is owned by the lake's part.  The lake's
 * stage is owned there; the reaches flowing into it are ghosts there if owned elsewhere (their QrivDown is
 * recomputed from the exchanged stage).  A rank's owned state is [sf|us|gw|riv|lake(owned)].
 */
#ifndef SHUD_PARTITION_H
#define SHUD_PARTITION_H

#include <stdint.h>

#include "shud_rhs.h"

#ifdef __cplusplus
extern "C" {
#endif

#define SHUD_PART_MULTILEVEL 0
#define SHUD_PART_RCB        1
#define SHUD_PART_AUTO       2   /* multilevel, and RCB when centroids are given: the smaller largest halo */
#define SHUD_PART_MAX_PARTS  64

typedef struct ShudPartStats {
    int64_t edge_cut;        /* mesh edges whose two elements lie on different parts                     */
    int64_t segment_cut;     /* river segments whose element and reach are owned by different parts      */
    int64_t graph_cut;       /* weighted cut of the multilevel graph (mesh + river coupling edges); -1 RCB */
    double  imbalance;       /* max part vertex weight / (total / nparts)                               */
    int32_t levels;          /* coarsening levels (multilevel)                                           */
    int32_t coarse_vertices; /* vertices of the coarsest graph                                           */
    double  seconds;         /* wall time of shud_partition_mesh                                         */
    int64_t max_halo;        /* largest per-part ghost count (ghost elements + ghost reaches)            */
    int32_t method_used;     /* SHUD_PART_MULTILEVEL or SHUD_PART_RCB (AUTO reports its pick)            */
} ShudPartStats;

/* Partition the elements of `mesh` into nparts (1..64).  cx/cy: element centroids (RCB only; may be NULL
 * for the multilevel method).  Deterministic for a given seed.  ele_part[NE] receives the part ids. */
int shud_partition_mesh(const ShudMeshSoA *mesh, const double *cx, const double *cy, int32_t nparts,
                        int32_t method, uint64_t seed, int32_t *ele_part, ShudPartStats *stats);
/* move every lake group of a caller's partition to one part (the part holding most of the group's vertex
 * weight; lowest on ties) — what shud_partition_mesh applies to its own result.  No-op without lakes. */
int shud_partition_constrain(const ShudMeshSoA *mesh, int32_t nparts, int32_t *ele_part);
/* edge/segment cut of any given element partition (same definitions as ShudPartStats) */
int shud_partition_cut(const ShudMeshSoA *mesh, const int32_t *ele_part, int32_t nparts, int64_t *edge_cut,
                       int64_t *segment_cut);

/* ghost elements / ghost reaches each part would hold (the halo one RHS exchanges) */
int shud_partition_halo(const ShudMeshSoA *mesh, const int32_t *ele_part, int32_t nparts, int64_t *ghost_ele,
                        int64_t *ghost_riv);

typedef struct shud_plan *shud_plan_t;

/* Build rank `rank`'s plan from an element partition (all ranks compute the same global ownership). */
int shud_plan_build(const ShudMeshSoA *mesh, const int32_t *ele_part, int32_t nparts, int32_t rank,
                    shud_plan_t *out);   /* SHUD_ERR_UNSUPPORTED: a lake group split across parts */
void shud_plan_free(shud_plan_t p);

typedef struct ShudPlanInfo {
    int32_t n_own_ele, n_int_ele, n_ghost_ele;   /* n_int: owned elements reading no ghost data (prefix)   */
    int32_t n_own_riv, n_ghost_riv, n_seg;
    const int32_t *ele_gid;   /* [n_own_ele + n_ghost_ele] global element of each local element           */
    const int32_t *riv_gid;   /* [n_own_riv + n_ghost_riv]                                                */
    const int32_t *seg_gid;   /* [n_seg] global segment of each local segment (ascending)                 */
    const int32_t *riv_part;  /* [NR global] reach owners                                                 */
    int32_t n_own_lake;       /* lakes owned by this rank (their stages follow the owned reaches in y)     */
    const int32_t *lake_gid;  /* [n_own_lake] global lake index (0-based) of each local lake, ascending    */
} ShudPlanInfo;
int shud_plan_info(shud_plan_t p, ShudPlanInfo *info);
/* ShudPartition for shud_rhs_create_partitioned; nccl_unique_id is left NULL (set it before create) */
int shud_plan_partition(shud_plan_t p, ShudPartition *part);
/* The rank's local mesh and parameters gathered from the global ones (arrays owned by the plan, valid until
 * shud_plan_free).  A local reach whose downstream reach is not local gets outlet code -3 (its QrivDown is
 * never used: only owned reaches' DY are computed and their downstream is always local).  Lakes: the owned
 * lakes, renumbered 1..n_own_lake in ilake / riv_down (-3 - id); a reach flowing into a lake owned elsewhere
 * gets the outlet code -3 (the same zero-depth-gradient QrivDown, MD_RiverFlux.cpp:17-25). */
int shud_plan_local_mesh(shud_plan_t p, const ShudMeshSoA *gmesh, const ShudParamsSoA *gpar, ShudMeshSoA *lmesh,
                         ShudParamsSoA *lpar);
/* gather a per-element global array [NE] into local order [n_own_ele + n_ghost_ele] (step inputs, carried
 * state, ET statics: ghosts carry replicated values) */
int shud_plan_gather_ele(shud_plan_t p, const double *global, double *local);
int shud_plan_gather_ele_i32(shud_plan_t p, const int32_t *global, int32_t *local);
/* owned block of a global state vector: [sf|us|gw|riv|lake](global) -> [sf|us|gw|riv|lake](owned, local order) */
int shud_plan_owned_state(shud_plan_t p, const double *y_global, int32_t ne_global, double *y_owned);
/* scatter an owned block back into a global vector (tests / gathers of a distributed result) */
int shud_plan_scatter_owned(shud_plan_t p, const double *y_owned, int32_t ne_global, double *y_global);

const char *shud_partition_error(void);

#ifdef __cplusplus
}
#endif
#endif /* SHUD_PARTITION_H */
