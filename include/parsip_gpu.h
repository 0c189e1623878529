/*
 * parsip_gpu.h — C-ABI of the MI355X (gfx950) BlobTree polygonizer.
 *
 * Drop-in boundary for Parsip's PS_SimdPoly hot path.  Every struct below is
 * byte-identical to the reference SoA contract so a host that fills
 * PS::SIMDPOLY::SOABlobPrims / SOABlobOps / SOABlobPrimMatrices can hand the
 * same bytes to this library:
 *
 *   reference struct                          (Parsip100/PS_SimdPoly/include/)
 *   SOABlobPrims        9,500 B  align 4      PS_Polygonizer.h:98-130
 *   SOABlobOps          5,636 B  align 4      PS_Polygonizer.h:134-154
 *   SOABlobPrimMatrices 6,148 B  align 4      PS_Polygonizer.h:161-165
 *   SOABlobBoxMatrices  8,196 B  align 4      PS_Polygonizer.h:171-175
 *   MPU                21,524 B  align 4      PS_Polygonizer.h:183-195
 *
 * Entry points (each one cites the reference interface it replaces):
 *   psgpu_count_mpus        <- CountMPUNeeded   PS_Polygonizer.h:384, .cpp:388-412
 *   psgpu_prepare_bboxes    <- PrepareBBoxes    PS_Polygonizer.h:385, .cpp:55-309
 *   psgpu_polygonize_mpus   <- Polygonize       PS_Polygonizer.h:386-391, .cpp:315-385
 *                              (blocking, fills the caller's PolyMPUs layout)
 *   psgpu_create/destroy/set_model/polygonize/finish/...
 *                           <- the same Polygonize split into a device-resident,
 *                              stream-ordered form (compact mesh stays in HBM)
 *   psgpu_translate_blobtree_type <- enum map for SimdPoly::linearizeBlobTree
 *                              (PS_HighPerformanceRender.cpp:42-364; _constSettings.h:26-38)
 *
 * Error codes keep PS_Polygonizer.h:47-50 and add explicit overflow / device codes
 * (the reference truncates at MAX_MPU_COUNT with only a printf, .cpp:355-356, and
 * never checks the 512 vertex / triangle per-MPU capacity, .cpp:785-824).
 *
 * No torch / HIP types appear in these signatures: streams are passed as void*
 * (a hipStream_t, NULL = the context's own stream).
 */
#ifndef PARSIP_GPU_H
#define PARSIP_GPU_H

#ifdef __HIPCC_RTC__  /* embedded in run-time compiled compat kernels: no system headers */
typedef __SIZE_TYPE__ size_t;
#ifndef offsetof
#define offsetof(t, m) __builtin_offsetof(t, m)
#endif
#else
#include <stddef.h>
#include <stdint.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* ---- constants (PS_Polygonizer.h:21-81) ---------------------------------- */
#define PSGPU_GRID_DIM              8      /* corners per MPU axis (GRID_DIM_8)   */
#define PSGPU_CELLS_PER_MPU         7
#define PSGPU_ISO_VALUE             0.5f
#define PSGPU_ISO_DIST              0.45420206f
#define PSGPU_NORMAL_DELTA          0.001f
#define PSGPU_MIN_CELL_SIZE         0.01f
#define PSGPU_MAX_TREE_NODES        128
#define PSGPU_PRIM_MATRIX_STRIDE    12
#define PSGPU_BOX_MATRIX_STRIDE     16
#define PSGPU_MAX_MPU_COUNT         24000  /* the reference PolyMPUs capacity     */
#define PSGPU_MAX_MPU_VERTEX_COUNT  512
#define PSGPU_MAX_MPU_TRIANGLE_COUNT 512

/* ---- return codes -------------------------------------------------------- */
#define PSGPU_RET_SUCCESS          1   /* RET_SUCCESS                              */
#define PSGPU_RET_PARAM_ERROR     -1   /* RET_PARAM_ERROR (ctPrims == 0, bad args) */
#define PSGPU_RET_NOT_ENOUGH_MEM  -2   /* RET_NOT_ENOUGH_MEM (device alloc failed)  */
#define PSGPU_RET_INVALID_BVH     -3   /* RET_INVALID_BVH (op tree not a tree)      */
#define PSGPU_RET_MPU_OVERFLOW    -4   /* more MPUs than the caller's capacity      */
#define PSGPU_RET_MPU_VT_OVERFLOW -5   /* an MPU exceeds 512 vertices / triangles   */
#define PSGPU_RET_DEVICE_ERROR    -6   /* HIP / RCCL runtime error                  */

/* ---- node types: the hot path's own ordering (PS_Polygonizer.h:84-91) ---- */
enum PsNodeType {
    PSGPU_PRIM_CYLINDER = 0, PSGPU_PRIM_DISC = 1, PSGPU_PRIM_LINE = 2, PSGPU_PRIM_POINT = 3,
    PSGPU_PRIM_RING = 4, PSGPU_PRIM_POLYGON = 5, PSGPU_PRIM_CUBE = 6, PSGPU_PRIM_TRIANGLE = 7,
    PSGPU_PRIM_CATMULLROM = 8, PSGPU_PRIM_SKELETON = 9, PSGPU_PRIM_QUADRICPOINT = 10,
    PSGPU_PRIM_FASTQPS = 11, PSGPU_PRIM_HALFPLANE = 12, PSGPU_PRIM_NULL = 13,
    PSGPU_OP_UNION = 14, PSGPU_OP_INTERSECT = 15, PSGPU_OP_DIF = 16, PSGPU_OP_SMOOTHDIF = 17,
    PSGPU_OP_BLEND = 18, PSGPU_OP_RICCIBLEND = 19, PSGPU_OP_GRADIENTBLEND = 20,
    PSGPU_OP_AFFINE = 21, PSGPU_OP_WARPTWIST = 22, PSGPU_OP_WARPTAPER = 23,
    PSGPU_OP_WARPBEND = 24, PSGPU_OP_WARPSHEAR = 25, PSGPU_OP_CACHE = 26,
    PSGPU_OP_TEXTURE = 27, PSGPU_OP_PCM = 28
};

/* ---- SoA model (byte-exact) ---------------------------------------------- */
typedef struct PsVec3f { float x, y, z; } PsVec3f;

typedef struct PsSoaBlobPrims {          /* SOABlobPrims, PS_Polygonizer.h:98-130 */
    float posX[128], posY[128], posZ[128];
    float dirX[128], dirY[128], dirZ[128];
    float resX[128], resY[128], resZ[128];
    float colorX[128], colorY[128], colorZ[128];
    float vPrimBoxLoX[128], vPrimBoxLoY[128], vPrimBoxLoZ[128];
    float vPrimBoxHiX[128], vPrimBoxHiY[128], vPrimBoxHiZ[128];
    uint8_t skeletType[128];
    uint8_t idxMatrix[128];
    PsVec3f bboxLo;
    PsVec3f bboxHi;
    uint32_t ctPrims;
} PsSoaBlobPrims;

typedef struct PsSoaBlobOps {            /* SOABlobOps, PS_Polygonizer.h:134-154 */
    uint8_t opType[128];
    uint8_t opLeftChild[128];
    uint8_t opRightChild[128];
    uint8_t opChildKind[128];            /* bit1: left is op, bit0: right is op  */
    float vBoxLoX[128], vBoxLoY[128], vBoxLoZ[128];
    float vBoxHiX[128], vBoxHiY[128], vBoxHiZ[128];
    float resX[128], resY[128], resZ[128], resW[128];
    uint32_t ctOps;
} PsSoaBlobOps;

typedef struct PsSoaPrimMatrices {       /* SOABlobPrimMatrices, :161-165 (row 0 = identity) */
    float matrix[128 * PSGPU_PRIM_MATRIX_STRIDE];
    uint32_t count;
} PsSoaPrimMatrices;

typedef struct PsSoaBoxMatrices {        /* SOABlobBoxMatrices, :171-175 */
    float matrix[128 * PSGPU_BOX_MATRIX_STRIDE];
    uint32_t count;
} PsSoaBoxMatrices;

typedef struct PsMPU {                   /* MPU, PS_Polygonizer.h:183-195 */
    float vPos[PSGPU_MAX_MPU_VERTEX_COUNT * 3];
    float vNorm[PSGPU_MAX_MPU_VERTEX_COUNT * 3];
    float vColor[PSGPU_MAX_MPU_VERTEX_COUNT * 3];
    uint16_t triangles[PSGPU_MAX_MPU_TRIANGLE_COUNT * 3];
    uint16_t ctVertices;
    uint16_t ctTriangles;
    PsVec3f bboxLo;
    uint32_t ctFieldEvals;
} PsMPU;

/* Per-MPU outcome of a run (the library's own record; the reference's MPUSTATS is
 * PsMpuProcessStats below -- a different layout). */
typedef struct PsMpuStats {
    uint32_t passedPrecheck;   /* S1 (8-corner F>0 test) passed                  */
    uint32_t ctFieldEvals;     /* 128 if S1 passed else 0 (reference counter)     */
    uint32_t ctVertices;
    uint32_t ctTriangles;
} PsMpuStats;

/* MPUSTATS (PS_Polygonizer.h:201-207) in the reference's LP64 layout: int idxThread,
 * int bIntersected, tbb_thread::id threadID (a pthread_t), tbb::tick_count tickStart,
 * tickEnd (one long long each: legacy TBB's tick_count::now() on Linux is CLOCK_REALTIME in
 * nanoseconds).  CMPUProcessor::operator() (.cpp:449-461) writes threadID, tickStart and
 * tickEnd of every MPU and leaves idxThread / bIntersected alone; so does the library
 * (psgpu_download_process_stats):
 *   tickStart  the start of the wavefront that ran the MPU's S1 (k_precheck),
 *   tickEnd    the end of the wavefront that ran its S2-S3 and made its vertex / triangle
 *              records (k_mpu), or of its S1 wave when no S2 was needed (S1 failed, or field
 *              bounds proved it surface-free); S4-S6 run batched over every MPU's records in
 *              k_vertex / k_finish (psgpu_last_kernel_times gives their spans),
 *   threadID   the hardware slot of that last wave: XCC_ID << 16 | HW_ID[15:0] (wave slot,
 *              SIMD, CU, SH, SE), the device's "thread",
 * both ticks in CLOCK_REALTIME nanoseconds, mapped from the device clock (s_memrealtime)
 * by bracketing one device clock reading with the host clock (a few microseconds). */
typedef struct PsMpuProcessStats {
    int32_t  idxThread;
    int32_t  bIntersected;
    uint64_t threadID;
    int64_t  tickStart;
    int64_t  tickEnd;
} PsMpuProcessStats;

/* Result summary of one polygonization. */
typedef struct PsMeshInfo {
    uint32_t ctMPUs;            /* MPUs in the processed range                     */
    uint32_t ctPassedPrecheck;  /* MPUs that passed S1                              */
    uint32_t ctSurfaceMPUs;     /* MPUs that produced >= 1 triangle                 */
    uint32_t ctVertices;
    uint32_t ctTriangles;
    int32_t  firstOverflowMPU;  /* global MPU id with > 512 V or T, or -1           */
    uint64_t ctLaneEvals;       /* field evaluations performed (per point)          */
    uint32_t ctFieldMPUs;       /* S1 survivors whose 8^3 field cache was evaluated
                                 * (the rest were proven empty by field bounds)     */
    uint32_t launchFlags;       /* how the run was launched: PSGPU_LAUNCH_*         */
} PsMeshInfo;
#define PSGPU_LAUNCH_TREE_SPLIT 1u  /* k_precheck / k_mpu walked the root's subtrees in two waves */
#define PSGPU_LAUNCH_SURFACE    2u  /* k_vertex + k_finish ran as one launch (k_surface)         */
#define PSGPU_LAUNCH_FRONT      4u  /* k_precheck + k_mpu ran as one launch (k_front)            */
#define PSGPU_LAUNCH_RERUN      8u  /* finish re-ran the run (grid / capacity / protocol error)  */

/* Device-resident compact mesh of the last polygonization (pointers into the
 * context's HBM buffers; valid until the next psgpu_polygonize on the context).
 * The vertices of the w-th MPU of the processed range [mpuBegin, mpuEnd) occupy
 * [(uint32)mpuOffsets[w], (uint32)mpuOffsets[w+1]) and its triangles
 * [mpuOffsets[w] >> 32, mpuOffsets[w+1] >> 32): MPU order, i.e. exactly the reference's
 * concatenation of vMPUs[i].vPos / triangles over i (PS_Polygonizer.cpp:360-371).   */
typedef struct PsMeshDevice {
    const float*    pos;              /* ctVertices * 3, xyz interleaved           */
    const float*    nrm;              /* ctVertices * 3                            */
    const float*    col;              /* ctVertices * 3                            */
    const uint32_t* tris;             /* ctTriangles * 3, global vertex ids        */
    const uint64_t* mpuOffsets;       /* ctMPUs + 1, exclusive scan:
                                         vertexOffset | triangleOffset << 32      */
} PsMeshDevice;

typedef struct psgpu_ctx psgpu_ctx;

/* ---- host-only helpers --------------------------------------------------- */
/* CountMPUNeeded (PS_Polygonizer.cpp:388-412). */
uint32_t psgpu_count_mpus(float cellsize, const float lo[3], const float hi[3]);
/* MPU lattice dimensions along x,y,z (PS_Polygonizer.cpp:339-352). */
int psgpu_mpu_dims(float cellsize, const PsSoaBlobPrims* prims, uint32_t dims[3]);
/* PrepareBBoxes (PS_Polygonizer.cpp:55-309) with the exact iso distance
 * PSGPU_ISO_DIST instead of the reference's undefined-behaviour FastSqrt. */
int psgpu_prepare_bboxes(float cellsize, PsSoaBlobPrims* prims, PsSoaBoxMatrices* boxMatrices,
                         PsSoaBlobOps* ops);
/* _constSettings.h:26-38 code (caller / PS_BlobTree side) -> PsNodeType; -1 if none. */
int psgpu_translate_blobtree_type(int blobtreeType);
/* Marching-cubes triangle table (256 x 16, -1 padded), generated at load time. */
void psgpu_tritable(int32_t out[256 * 16]);
/* Library version string. */
const char* psgpu_version(void);

/* ---- device context ------------------------------------------------------ */
int  psgpu_create(int deviceOrdinal, psgpu_ctx** out);
/* Frees the context; waits for an in-flight compile of its model's kernels first (call
 * it before the process exits: a compile must not run while the process tears down). */
void psgpu_destroy(psgpu_ctx* ctx);
int  psgpu_device_count(void);
/* Upload a model (validates the op tree; builds the device walk program). */
int  psgpu_set_model(psgpu_ctx* ctx, const PsSoaBlobPrims* prims,
                     const PsSoaPrimMatrices* matrices, const PsSoaBlobOps* ops);
/* Enqueue a polygonization of global MPUs [mpuBegin, mpuEnd) (clamped to the
 * lattice; pass 0, UINT32_MAX for all) on `stream` (hipStream_t or NULL). Async.
 * A range (after clamping) holds fewer than 2^26 MPUs (a 4096^3-cell lattice is 2^27:
 * split it into ranges); a larger one returns PSGPU_RET_PARAM_ERROR. */
int  psgpu_polygonize(psgpu_ctx* ctx, float cellsize, uint32_t mpuBegin, uint32_t mpuEnd,
                      void* stream);
/* Wait for the last polygonize and report counts / errors.  If the output
 * buffers were too small the call re-runs the polygonization with grown buffers. */
int  psgpu_finish(psgpu_ctx* ctx, PsMeshInfo* info);
int  psgpu_mesh_device(psgpu_ctx* ctx, PsMeshDevice* out);
/* Copy the compact mesh to host arrays (any pointer may be NULL); mpuOffsets gets
 * ctMPUs + 1 entries as in PsMeshDevice. */
int  psgpu_download_mesh(psgpu_ctx* ctx, float* pos, float* nrm, float* col, uint32_t* tris,
                         uint64_t* mpuOffsets);
/* Per-MPU stats for every MPU in the last processed range (ctMPUs entries). */
int  psgpu_download_stats(psgpu_ctx* ctx, PsMpuStats* stats);
/* Scatter the last result into the reference PolyMPUs layout (vMPUs[0..ctMPUs)). */
int  psgpu_export_polympus(psgpu_ctx* ctx, PsMPU* mpus, uint32_t capacity, uint32_t* outCtMPUs);
/* Blocking drop-in for PS::SIMDPOLY::Polygonize: upload, run, export. */
int  psgpu_polygonize_mpus(psgpu_ctx* ctx, float cellsize, const PsSoaBlobPrims* prims,
                           const PsSoaPrimMatrices* matrices, const PsSoaBlobOps* ops,
                           PsMPU* mpus, uint32_t capacity, uint32_t* outCtMPUs,
                           PsMpuStats* statsOrNull);
/* The same with the reference's MPUSTATS* lpProcessStats (Polygonize :386-391, :379): when
 * processStats is not NULL the run records per-MPU ticks (PSGPU_OPT_MPU_TICKS for this call)
 * and processStats[0..ctMPUs) receives them as psgpu_download_process_stats gives them. */
int  psgpu_polygonize_mpus_ex(psgpu_ctx* ctx, float cellsize, const PsSoaBlobPrims* prims,
                              const PsSoaPrimMatrices* matrices, const PsSoaBlobOps* ops,
                              PsMPU* mpus, uint32_t capacity, uint32_t* outCtMPUs,
                              PsMpuStats* statsOrNull, PsMpuProcessStats* processStatsOrNull);
/* MPUSTATS of the last run (ctMPUs entries; threadID, tickStart, tickEnd written, the other
 * fields untouched, as the reference).  PSGPU_RET_PARAM_ERROR if that run did not record
 * ticks (PSGPU_OPT_MPU_TICKS was 0 when it was enqueued). */
int  psgpu_download_process_stats(psgpu_ctx* ctx, PsMpuProcessStats* out);
/* Per-wave timeline of the last polygonize (PSGPU_OPT_STAMPS > 0; the reference's
 * MPUSTATS / PrintThreadResults, PS_Polygonizer.h:201-207, .cpp:414-461, with waves for
 * threads): 4 kernels (precheck, mpu, vertex, finish) x cap records of 3 uint64:
 * start, end (100 MHz s_memrealtime ticks), item | hw id << 32 where item is the MPU a
 * k_mpu wave polygonized (0xffffffff: none) or the wave's index, hw id = HW_ID[15:0] |
 * XCC_ID << 16.  Unlaunched waves read zero; then cap x 8 words of k_mpu phase stamps
 * (PSGPU_OPT_DEBUG bit 4096; profiling only).  Pass out = NULL to query *cap. */
int  psgpu_download_stamps(psgpu_ctx* ctx, uint64_t* out, uint32_t* cap);
/* PrintThreadResults (PS_Polygonizer.h:393, body .cpp:414-428, counters .cpp:443-469).
 * The reference keeps one (processed, crossed) MPU count pair per TBB worker that ran an
 * MPU, accumulated over every Polygonize of the process.  Here the worker is a device
 * context: every finished run (psgpu_finish, and every call built on it: the blocking
 * psgpu_polygonize_mpus, group parts, comm ranks) adds the MPUs of its range and those with
 * ctTriangles > 0 to its context's entry; entries are enumerated in the order contexts first
 * finished a run and outlive their context.  This divides each entry by ctAttempts, stores
 * entry i into lpThreadProcessed[i] / lpThreadCrossed[i] (either may be NULL; at most
 * `capacity` entries are written: pass psgpu_thread_result_count()), prints
 * "Thread#  i, Processed MPUs p, Crossed MPUs c " lines as the reference when print != 0,
 * clears every entry, and returns the number of entries.  ctAttempts <= 0:
 * PSGPU_RET_PARAM_ERROR, nothing cleared. */
int  psgpu_print_thread_results(int ctAttempts, uint32_t* lpThreadProcessed, uint32_t* lpThreadCrossed,
                                uint32_t capacity, int print);
/* Entries psgpu_print_thread_results would report now. */
int  psgpu_thread_result_count(void);
/* Device-side timing of the last polygonize, per kernel (ms); returns count filled. */
int  psgpu_last_kernel_times(psgpu_ctx* ctx, float* ms, int maxKernels, const char** names);
/* FieldComputer::fieldValue / fieldValueAndColor on n host points (xyz interleaved):
 * mode 0 = consecutive points form the reference's 4-lane pruning groups,
 * mode 1 = every point alone (4 identical lanes), mode 2 = mode 1 + colour (n*3). */
int  psgpu_field_values(psgpu_ctx* ctx, const float* xyz, uint32_t n, int mode, float* out, float* colOut);
/* Kernel spans of the runs recorded since PSGPU_OPT_SPANS was set: *runs slots of
 * 4 kernels x {start, end} (s_memrealtime, 100 MHz); out = NULL queries *runs. */
int  psgpu_download_spans(psgpu_ctx* ctx, uint64_t* out, uint32_t* runs);

/* Set a context option (see PSGPU_OPT_*). */
int  psgpu_set_option(psgpu_ctx* ctx, int option, int64_t value);
#define PSGPU_OPT_KERNEL_TIMING 1   /* 1: record hipEvents around every kernel */
#define PSGPU_OPT_CULLING       2   /* 1: exact per-wave primitive culling (default) */
#define PSGPU_OPT_DEBUG         9   /* profiling ablations (bit 0: stop after S2); 0 in use;
                                       bit 20 (test hook): the next run's k_mpu grid is one
                                       block, so finish must re-run it with the full grid;
                                       bits 23 / 24 (test hooks of the blocking export): the
                                       staging past the piece flags is filled with the call's
                                       epoch before the export / the packing kernel's last
                                       block waits ~40 us before each piece;
                                       bits 25 / 26 / 27 (test hooks, the next run only):
                                       k_surface's scan blocks count themselves done ~40 us
                                       late and its waves give up waiting after a few spins /
                                       every offsets-scan look-back times out / k_front's S1
                                       blocks publish ~40 us late and its S2 waves give up
                                       after a few polls; either way finish sees the protocol
                                       error and re-runs the polygonization as separate
                                       launches (k_precheck, k_mpu, k_vertex, k_finish; a
                                       second error: -6);
                                       bit 28 (test hook): the next run starts 3 runs short of
                                       the run counter's 32-bit wrap, where the context
                                       restarts its counter sets at epoch 0 */
#define PSGPU_OPT_VERTEX_BLOCKS_PER_CU 4  /* persistent k_vertex grid, 256-thread blocks per CU; once a
                                             run of the same range has finished, the grid is fitted
                                             to its vertices (+1/8) up to this (env PSGPU_GRID_FIT=0:
                                             always the persistent grid) */
#define PSGPU_OPT_FINISH_BLOCKS_PER_CU 5  /* persistent k_finish grid (fitted the same way) */
#define PSGPU_OPT_GRAPH         7   /* 1: replay repeated launch sequences from a hipGraph (off by
                                       default: +4-5 us per polygonization on ROCm 7.2) */
#define PSGPU_OPT_CAPACITY      6   /* restart output buffers at this vertex capacity (>= 64;
                                       they grow and the run repeats when exceeded) */
#define PSGPU_OPT_BOUND        10   /* 1: k_precheck proves S1 survivors without a surface by
                                       conservative field bounds and skips their S2 (default;
                                       output unchanged; JIT kernels only) */
#define PSGPU_OPT_JIT           3   /* 0 interpreter, 1 specialised per structure (default),
                                       2 specialised with parameters baked in (a recompile per
                                       parameter change), 3 tiered: the structure kernels at once,
                                       then -- once the model has stayed unchanged for
                                       PSGPU_OPT_TIER_RUNS polygonizations -- its baked kernels,
                                       compiled on a host thread and swapped in when loaded; a
                                       set_model that changes the model returns to the structure
                                       kernels at once (no compile on an animation's frame path).
                                       Identical output in every mode */
#define PSGPU_OPT_TIER_RUNS    18   /* tier-up threshold of PSGPU_OPT_JIT 3 (default 16, >= 1) */
#define PSGPU_OPT_STAMPS       12   /* > 0: record a per-wave timeline for up to this many waves
                                       per kernel (psgpu_download_stamps); 0: off (default) */
#define PSGPU_OPT_SPANS        13   /* > 0: the next this-many runs record each kernel's span on the
                                       device clock (first wave start, last wave end; 100 MHz) */
#define PSGPU_OPT_FINISH_QUAD  14   /* k_finish layout: 0 one lane per vertex (64 per wave), 1 a quad
                                       of lanes per vertex (16 per wave), 3 a pair of lanes (32 per
                                       wave), 2 (default) the fewest vertices per wave whose waves
                                       hold the last run's vertices in one pass of the persistent
                                       grid (16 or 32; else 64: small rank shares), at most 32 for a
                                       run enqueued while no other context of the process has a run
                                       pending on the device (a blocking caller, one context queueing
                                       its frames); identical output */
#define PSGPU_OPT_VERTEX_WIDE  15   /* k_vertex layout: 0 a quad of lanes per vertex (16 per wave),
                                       1 one lane per vertex walking its 4 edge samples (64 per wave,
                                       specialised kernels only), 2 (default) 64 when the last run's
                                       vertices overfill one pass of the persistent grid at 16 per
                                       wave and other contexts of the process have runs pending on
                                       the device (contexts taking frames in turn), else 16;
                                       identical output */
#define PSGPU_OPT_TREE_SPLIT   16   /* 1: k_precheck and k_mpu walk the root's two subtrees in two
                                       waves per brick / MPU and combine them (specialised kernels,
                                       trees whose root is a binary op over two ops); 2: only for runs
                                       whose range queued at most PSGPU_OPT_SPLIT_MAX_QUEUED MPUs for
                                       S2 last time (small rank shares); 0 (default) one wave walks the
                                       whole tree.  Non-zero compiles the split kernels too (+30-45 %
                                       hiprtc time).  Identical output */
#define PSGPU_OPT_SPLIT_MAX_QUEUED 17  /* threshold of PSGPU_OPT_TREE_SPLIT 2 (default 4 per CU) */
#define PSGPU_OPT_FUSED_SURFACE 21  /* k_vertex + k_finish as one launch (quad layouts, the offsets
                                       scan released inside it): 2 (default) for runs whose last
                                       run's vertices take the quad layouts in both (small rank
                                       shares), 1 always, 0 never, 3 always with one lane per
                                       vertex for both walks (k_surface_w: full grids; measured
                                       within 1-2 % of the two launches, so not a default).  Needs
                                       the small-launch kernels, compiled with
                                       PSGPU_OPT_TREE_SPLIT != 0.  Identical output */
#define PSGPU_OPT_FRONT        22   /* k_precheck + k_mpu as one launch, S1 survivors handed to the
                                       S2 blocks of the same launch as they are published (no grid
                                       barrier): 0 two launches, 1 always (generated kernels),
                                       2 (default) when k_precheck's grid is at most 8 blocks per
                                       CU (C3 and its shares, not C5's 512^3 frame); env
                                       PSGPU_FRONT; never with PSGPU_OPT_MPU_TICKS, nor while
                                       more than 3 other contexts have runs pending on the device */
#define PSGPU_OPT_MPU_TICKS    19   /* 1: runs record per-MPU ticks for MPUSTATS
                                       (psgpu_download_process_stats); 0 (default) off */
#define PSGPU_OPT_JIT_ASYNC    11   /* 1 (default): set_model returns at once; hiprtc compiles the
                                       specialised kernels on a host thread while the interpreter
                                       serves polygonizations (bit-identical output); 0: block */
/* Host-only (no GPU): compile the model's specialised kernels with hiprtc (mode 1:
 * structure only, 2: parameters baked in; | 4: with the tree-split kernels); returns the
 * code-object size or a negative error (log receives the compiler output). */
long psgpu_jit_compile(const PsSoaBlobPrims* prims, const PsSoaPrimMatrices* matrices,
                       const PsSoaBlobOps* ops, int mode, char* log, size_t cap);
/* 1 if the current model runs on run-time specialised kernels, 0 on the interpreter. */
int  psgpu_jit_active(psgpu_ctx* ctx);
/* 1 while the current model's specialised kernels are still compiling. */
int  psgpu_jit_pending(psgpu_ctx* ctx);
/* Block until the current model's compile has finished and adopt its kernels (with
 * PSGPU_OPT_JIT 3 also a baked compile already started); returns psgpu_jit_active
 * afterwards (0: the compile failed and the interpreter stays). */
int  psgpu_jit_wait(psgpu_ctx* ctx);
/* The kernels the next run uses: 0 interpreter, 1 structure-specialised, 2 baked. */
int  psgpu_jit_tier(psgpu_ctx* ctx);
/* Generated specialised HIP source of the current model; returns its length. */
int  psgpu_jit_source(psgpu_ctx* ctx, char* buf, size_t cap);

/* Per-MPU work of the last run in lane-evaluations (8 S1 + 64 field bounds of a survivor
 * or 512 S2 cache of a queued survivor + 8 per vertex), ctMPUs entries. */
int  psgpu_mpu_costs(psgpu_ctx* ctx, uint32_t* costs);
/* Contiguous ranges of near-equal cost over n MPUs starting at global id `begin`:
 * bounds[0..parts] (bounds[0] = begin, bounds[parts] = begin + n).  Host only. */
int  psgpu_split_costs(const uint32_t* costs, uint32_t n, uint32_t parts, uint32_t begin,
                       uint32_t* bounds);

/* ---- one grid over several devices (one process) --------------------------
 * The reference's Polygonize fans the MPU list over every core in one blocking call
 * (tbb::parallel_for, PS_Polygonizer.cpp:379-382); a group fans one MPU lattice over
 * several GPUs: contiguous MPU ranges of near-equal cost, one context per device, every
 * device launched at once.  Parts concatenated in order are exactly the single-device
 * mesh (MPUs are independent: no halo).  Several parts may share a device. */
typedef struct psgpu_group psgpu_group;
typedef struct PsGroupPart {
    int32_t  device;          /* HIP ordinal (-1: another rank's device, psgpu_comm)  */
    uint32_t mpuBegin;        /* global MPU range [mpuBegin, mpuEnd)                  */
    uint32_t mpuEnd;
    uint32_t vertexBase;      /* first vertex / triangle of the part in the whole mesh */
    uint32_t triangleBase;
    uint32_t reserved;
    PsMeshInfo info;          /* the part's own counts                                 */
} PsGroupPart;

#define PSGPU_GROUP_OPT_BALANCE       100 /* range split policy (value below)           */
#define PSGPU_GROUP_BALANCE_EVEN        0 /* equal MPU counts                            */
#define PSGPU_GROUP_BALANCE_PLAN        1 /* cost split from a planning run of the whole
                                             lattice, redone when the lattice changes
                                             (default)                                  */
#define PSGPU_GROUP_BALANCE_EVERY_RUN   2 /* plan, then re-split after every finish from
                                             the costs of that run (animations)          */
#define PSGPU_GROUP_BALANCE_FIXED       3 /* the split of psgpu_group_set_split          */
#define PSGPU_GROUP_OPT_MIN_PART_MPUS 101 /* 0 (default): every part gets a range; n > 0:
                                             only the first max(1, lattice MPUs / n) parts
                                             do, the others stay empty -- a small lattice
                                             runs as one chain (EVEN / PLAN / EVERY_RUN) */

/* devices: nParts HIP ordinals (NULL: 0 .. nParts-1). */
int  psgpu_group_create(const int* devices, int nParts, psgpu_group** out);
void psgpu_group_destroy(psgpu_group* g);
int  psgpu_group_size(psgpu_group* g);
/* The context of one part (its device-resident part of the mesh, options, timing). */
psgpu_ctx* psgpu_group_context(psgpu_group* g, int part);
/* PSGPU_GROUP_OPT_BALANCE, or any PSGPU_OPT_* (applied to every part). */
int  psgpu_group_set_option(psgpu_group* g, int option, int64_t value);
int  psgpu_group_set_model(psgpu_group* g, const PsSoaBlobPrims* prims,
                           const PsSoaPrimMatrices* matrices, const PsSoaBlobOps* ops);
int  psgpu_group_jit_wait(psgpu_group* g);
/* Explicit split: bounds[0..nParts] global MPU ids, non-decreasing (policy FIXED). */
int  psgpu_group_set_split(psgpu_group* g, const uint32_t* bounds);
int  psgpu_group_get_split(psgpu_group* g, uint32_t* bounds);
/* Enqueue the whole lattice over the parts (asynchronous on every device). */
int  psgpu_group_polygonize(psgpu_group* g, float cellsize);
/* Wait for every part; totals over the parts and, if parts != NULL, nParts entries. */
int  psgpu_group_finish(psgpu_group* g, PsMeshInfo* total, PsGroupPart* parts);
/* The whole mesh to host arrays (global vertex ids and MPU offsets, as one device). */
int  psgpu_group_download_mesh(psgpu_group* g, float* pos, float* nrm, float* col, uint32_t* tris,
                               uint64_t* mpuOffsets);
/* The whole mesh in HBM of part dstPart's device (peer copies over xGMI + rebase). */
int  psgpu_group_gather(psgpu_group* g, int dstPart, PsMeshDevice* out);
int  psgpu_group_export_polympus(psgpu_group* g, PsMPU* mpus, uint32_t capacity, uint32_t* outCtMPUs);
/* Blocking drop-in for PS::SIMDPOLY::Polygonize over every device of the group. */
int  psgpu_group_polygonize_mpus(psgpu_group* g, float cellsize, const PsSoaBlobPrims* prims,
                                 const PsSoaPrimMatrices* matrices, const PsSoaBlobOps* ops,
                                 PsMPU* mpus, uint32_t capacity, uint32_t* outCtMPUs);

/* ---- one process per GPU: the count exchange over RCCL (xGMI) --------------
 * Every rank polygonizes its range of one split (psgpu_split_costs of the same costs on
 * every rank) on its own context; psgpu_comm_exchange all-gathers each rank's totals
 * (8 words, written by the run's last kernel) on the context's stream. */
typedef struct psgpu_comm psgpu_comm;
#define PSGPU_COMM_ID_BYTES 128
/* Rank 0 makes the id; the caller broadcasts its bytes to the other ranks. */
int  psgpu_comm_unique_id(uint8_t id[PSGPU_COMM_ID_BYTES]);
int  psgpu_comm_create(psgpu_ctx* ctx, const uint8_t id[PSGPU_COMM_ID_BYTES], int nranks, int rank,
                       psgpu_comm** out);
void psgpu_comm_destroy(psgpu_comm* comm);
/* Enqueue the all-gather of the context's last polygonization (after psgpu_polygonize). */
int  psgpu_comm_exchange(psgpu_comm* comm, psgpu_ctx* ctx);
/* The same for a rank whose range runs as a group of parts on its one device (several
 * streams): their totals are summed on part 0's stream before the all-gather. */
int  psgpu_comm_exchange_group(psgpu_comm* comm, psgpu_group* g);
/* Wait; totals over all ranks and, if parts != NULL, nranks entries (rank order).  A
 * collective: every rank calls it.  If any rank's finish re-ran its polygonization (grown
 * buffers), the ranks agree on that (all-reduce MAX of a flag) and all exchange again. */
int  psgpu_comm_result(psgpu_comm* comm, PsMeshInfo* total, PsGroupPart* parts);
/* 1 if the last psgpu_comm_result needed that second exchange (tests, diagnostics). */
int  psgpu_comm_reexchanged(psgpu_comm* comm);

#ifdef __cplusplus
} /* extern "C" */
#endif

#ifdef __cplusplus
static_assert(sizeof(PsSoaBlobPrims) == 9500, "SOABlobPrims size");
static_assert(offsetof(PsSoaBlobPrims, skeletType) == 9216, "skeletType offset");
static_assert(offsetof(PsSoaBlobPrims, idxMatrix) == 9344, "idxMatrix offset");
static_assert(offsetof(PsSoaBlobPrims, bboxLo) == 9472, "bboxLo offset");
static_assert(offsetof(PsSoaBlobPrims, ctPrims) == 9496, "ctPrims offset");
static_assert(sizeof(PsSoaBlobOps) == 5636, "SOABlobOps size");
static_assert(offsetof(PsSoaBlobOps, vBoxLoX) == 512, "vBoxLoX offset");
static_assert(offsetof(PsSoaBlobOps, resX) == 3584, "resX offset");
static_assert(offsetof(PsSoaBlobOps, ctOps) == 5632, "ctOps offset");
static_assert(sizeof(PsSoaPrimMatrices) == 6148, "SOABlobPrimMatrices size");
static_assert(sizeof(PsSoaBoxMatrices) == 8196, "SOABlobBoxMatrices size");
static_assert(sizeof(PsMPU) == 21524, "MPU size");
static_assert(offsetof(PsMPU, vNorm) == 6144, "vNorm offset");
static_assert(offsetof(PsMPU, vColor) == 12288, "vColor offset");
static_assert(offsetof(PsMPU, triangles) == 18432, "triangles offset");
static_assert(offsetof(PsMPU, ctVertices) == 21504, "ctVertices offset");
static_assert(offsetof(PsMPU, bboxLo) == 21508, "MPU bboxLo offset");
static_assert(offsetof(PsMPU, ctFieldEvals) == 21520, "ctFieldEvals offset");
static_assert(sizeof(PsMpuProcessStats) == 32, "MPUSTATS size (LP64)");
static_assert(offsetof(PsMpuProcessStats, threadID) == 8, "MPUSTATS threadID offset");
static_assert(offsetof(PsMpuProcessStats, tickStart) == 16, "MPUSTATS tickStart offset");
static_assert(offsetof(PsMpuProcessStats, tickEnd) == 24, "MPUSTATS tickEnd offset");
#else
_Static_assert(sizeof(PsSoaBlobPrims) == 9500, "SOABlobPrims size");
_Static_assert(sizeof(PsSoaBlobOps) == 5636, "SOABlobOps size");
_Static_assert(sizeof(PsSoaPrimMatrices) == 6148, "SOABlobPrimMatrices size");
_Static_assert(sizeof(PsSoaBoxMatrices) == 8196, "SOABlobBoxMatrices size");
_Static_assert(sizeof(PsMPU) == 21524, "MPU size");
#endif

#endif /* PARSIP_GPU_H */
