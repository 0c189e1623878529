/* parsip_gpu_gui.h -- C-ABI of the MI355X compat mode for ParsipHaptics' own polygonizer
 * ("GUI-path semantics").
 *
 * The GUI polygonizes with CParsipOptimized over a COMPACTBLOBTREE
 * (ParsipHaptics/include/CPolyParsipOptimized.{h,cpp}, CompactBlobTree.{h,cpp}) instead of
 * PS_SimdPoly.  It shares the MPU scheme (8^3 corners, 7^3 cells per MPU) but not its
 * semantics:
 *   - inside test `f > iso` (CPolyParsipOptimized.cpp:242; SIMD path: >=);
 *   - no S1 precheck: an MPU is processed when its box meets any primitive's octree
 *     (:164-183), all 512 corners are evaluated (lazy cache, :226-244);
 *   - vertices by ComputeRootNewtonRaphsonVEC4 (CompactBlobTree.cpp:1581-1622), normals by
 *     -1/delta central differences (:433-450), colours by baseColor over the field values
 *     stored by the last Newton evaluation (:1095-1294);
 *   - the field: n-ary operators, Ricci blend with powf, per-node backward matrices,
 *     warps (bend, twist, taper, shear), PCM contact and Instance nodes, no op-box
 *     pruning (:677-1092).
 * Every entry point below replaces the reference function named beside it.  The tree is
 * passed as the COMPACTBLOBTREE arrays (CompactBlobTree.h:26-61) with the per-operator
 * kid lists flattened into one array.  No CPU fallback: without a device every compute
 * call returns PSGPU_RET_DEVICE_ERROR.
 */
#ifndef PARSIP_GPU_GUI_H
#define PARSIP_GPU_GUI_H

#include "parsip_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Node types: the caller-side BlobNodeType enum (_constSettings.h:26-38). */
#define PSGUI_PRIM_POINT        0
#define PSGUI_PRIM_LINE         1
#define PSGUI_PRIM_CYLINDER     2
#define PSGUI_PRIM_DISC         3
#define PSGUI_PRIM_RING         4
#define PSGUI_PRIM_CUBE         6
#define PSGUI_PRIM_TRIANGLE     7
#define PSGUI_PRIM_QUADRICPOINT 10
#define PSGUI_PRIM_NULL         12
#define PSGUI_PRIM_INSTANCE     13   /* res1 = (origin's compact id, origin orgID, origin
                                        isOp, origin type): CompactBlobTree.cpp:383-391,
                                        resolved by updateInstanceNodes (:410-431)        */
#define PSGUI_OP_UNION          14
#define PSGUI_OP_INTERSECT      15
#define PSGUI_OP_DIF            16
#define PSGUI_OP_SMOOTHDIF      17
#define PSGUI_OP_BLEND          18
#define PSGUI_OP_RICCIBLEND     19
#define PSGUI_OP_PCM            22
#define PSGUI_OP_WARPTWIST      24
#define PSGUI_OP_WARPTAPER      25
#define PSGUI_OP_WARPBEND       26
#define PSGUI_OP_WARPSHEAR      27

#define PSGUI_MAX_DEPTH         32   /* operator nesting the device walk supports        */
#define PSGUI_GRID_DIM          8    /* GRID_DIM (CPolyParsipOptimized.h:23, GRID_DIM_8)  */
#define PSGUI_ITERATIONS        8    /* DEFAULT_ITERATIONS (_constSettings.h:8)           */
#define PSGUI_RET_UNSUPPORTED  -7    /* a tree the device walk does not evaluate: an operator
                                        without children, nesting > PSGUI_MAX_DEPTH (an
                                        Instance's origin subtree counted where the Instance
                                        sits), a PCM without exactly 2 kids (the reference
                                        returns 0 and reads an uninitialised kid colour),
                                        a PCM inside a PCM's kid subtree (also through an
                                        Instance), an Instance of a subtree holding an
                                        Instance (nested instancing; this also excludes
                                        cycles)                                            */
#define PSGUI_PCM_MARCH_MAX     64   /* marchTowardNode's steps (CompactBlobTree.cpp:572-592
                                        loops until |f - iso| < 1e-3, forever when it never
                                        gets there)                                        */

/* BlobPrimitive (CompactBlobTree.h:26-38); vec4f fields as float[4]. */
typedef struct PsGuiPrim {
    int32_t  type;
    int32_t  orgID;
    uint32_t idxMtx;     /* 0: identity; else a row of PsGuiMatrix                  */
    uint32_t reserved;
    float color[4];      /* material diffuse (rgba)                                 */
    float pos[4];
    float dir[4];
    float res1[4];
    float res2[4];
    float octLo[4];      /* the node's octree box (w unused)                         */
    float octHi[4];
} PsGuiPrim;

/* BlobOperator (CompactBlobTree.h:41-52): kids[kidStart .. kidStart + ctKids) of the
 * kid array, each (kid id) | (isOp << 16). */
typedef struct PsGuiOp {
    int32_t  type;
    int32_t  orgID;
    int32_t  ctKids;
    uint32_t kidStart;
    uint32_t idxMtx;
    uint32_t reserved[3];
    float params[4];     /* Ricci (n, 1/n); warps (factor / rate, axes, bend region) */
    float octLo[4];
    float octHi[4];
} PsGuiOp;

/* BlobNodeMatrix (CompactBlobTree.h:55-61): rows 0-3 of the backward matrix
 * (CMatrix::getRow); entry 0 is the identity. */
typedef struct PsGuiMatrix {
    float r[4][4];
} PsGuiMatrix;

/* CParsipOptimized's statistics (statsMeshInfo, statsIntersectedMPUs, statsTotalFieldEvals,
 * statsIntersectedCellsCount, countMPUs: CPolyParsipOptimized.cpp:487-527, .h:278-302). */
typedef struct PsGuiInfo {
    uint32_t dims[3];            /* the MPU lattice (setup, :348-365)                    */
    uint32_t ctLatticeMPUs;      /* MPUs created by setup                                */
    uint32_t ctMPUs;             /* countMPUs() after run(): removeExtraPUs (:403-405)   */
    uint32_t ctIntersectedMPUs;  /* statsIntersectedMPUs: MPUs with faces                */
    uint32_t ctProcessedMPUs;    /* MPUs whose box met a primitive's octree (:164-183)   */
    uint32_t ctVertices;
    uint32_t ctTriangles;
    uint32_t ctIntersectedCells; /* cells with config not 0 / 255 (:246-249)             */
    uint64_t ctFieldEvals;       /* statsTotalFieldEvals: cache + Newton + normal counts */
    uint64_t ctCellsInIntersectedMPUs; /* (GRID_DIM-1)^3 x intersected MPUs (.h:302)    */
} PsGuiInfo;

/* Per lattice MPU (CSIMDMPU statistics, CPolyParsipOptimized.h:60-117). */
typedef struct PsGuiMpuStats {
    uint32_t fieldEvals;
    uint32_t intersectedCells;
    uint32_t ctVertices;
    uint32_t ctTriangles;
} PsGuiMpuStats;

typedef struct psgpu_gui psgpu_gui;

int  psgpu_gui_create(int device, psgpu_gui** out);
void psgpu_gui_destroy(psgpu_gui* g);

/* The converted tree (COMPACTBLOBTREE::convert, CompactBlobTree.cpp:25-408): uploads it;
 * checks kid ids, depth and types (PSGUI_RET_UNSUPPORTED / PSGPU_RET_PARAM_ERROR). */
int  psgpu_gui_set_tree(psgpu_gui* g, const PsGuiPrim* prims, uint32_t ctPrims, const PsGuiOp* ops,
                        uint32_t ctOps, const uint32_t* kids, uint32_t ctKids, const PsGuiMatrix* mtx,
                        uint32_t ctMtx);

/* CParsipOptimized::setup + run (CPolyParsipOptimized.cpp:330-410): the lattice over the
 * root octree [octLo, octHi] at `cellsize`, polygonized at `isovalue`.  Stream-ordered;
 * psgpu_gui_finish waits. */
int  psgpu_gui_polygonize(psgpu_gui* g, const float octLo[3], const float octHi[3], float cellsize,
                          float isovalue);
int  psgpu_gui_finish(psgpu_gui* g, PsGuiInfo* info);

/* exportMesh (:594-613): the MPU meshes concatenated in lattice order; tris hold mesh-wide
 * vertex ids; colours are rgba.  mpuOffsets (ctLatticeMPUs + 1 entries, V | T << 32) and
 * stats (ctLatticeMPUs entries) may be NULL. */
int  psgpu_gui_download(psgpu_gui* g, float* pos, float* nrm, float* col4, uint32_t* tris,
                        uint64_t* mpuOffsets, PsGuiMpuStats* stats);

/* COMPACTBLOBTREE::fieldvalue and baseColor at n points (probe; col4 may be NULL).  PCM
 * nodes read the contact state below and never update it. */
int  psgpu_gui_field_values(psgpu_gui* g, const float* xyz, uint32_t n, float* out, float* col4);

/* The PCM contact state (PCMCONTEXT maxCompressionLeft / Right, CompactBlobTree.h:63-71),
 * one pair per tree shared by its PCM nodes, as the reference's.  The reference keeps it as
 * a running maximum that each TBB body's copy of the tree updates in its own evaluation
 * order (CompactBlobTree.cpp:508-521, a copy per body: CPolyParsipOptimized.h:171,188), so
 * its propagation fields depend on how TBB split the MPU range.  The defined order here:
 * a polygonization reads the state as it was when the run started (set_tree = convert sets
 * ISO_VALUE, :82-87: what every body of the reference starts from) and, when it ends,
 * raises the state to the largest compression any of its field evaluations met (the
 * corner cache, Newton steps and their gradient samples, normal samples -- exactly the
 * reference's evaluations).  get reads it (after finish); set replaces it
 * (stream-ordered, for the next run or probe). */
int  psgpu_gui_get_pcm_state(psgpu_gui* g, float state[2]);
int  psgpu_gui_set_pcm_state(psgpu_gui* g, const float state[2]);

/* Per-tree kernels.  set_tree starts compiling the tree's walk as straight-line code
 * (hiprtc, on a host thread; parameters stay in device memory, so only a structural edit
 * recompiles) while the interpreter kernels serve; polygonize swaps them in once loaded.
 * Both are bit-identical.  PSGUI_OPT_JIT: 0 interpreter only, 1 swap in when ready
 * (default; environment PSGUI_JIT overrides), 2 set_tree waits for the compile.
 * Trees with PCM or Instance nodes always run the interpreter's extended walk, without
 * culling (their sub-walks leave the wave's points: PCM marches toward a kid's surface, an
 * Instance evaluates its origin at its own point); their jit status stays NONE and
 * psgpu_gui_jit_compile returns PSGUI_RET_UNSUPPORTED for them. */
#define PSGUI_OPT_JIT           1
/* PSGUI_OPT_CULL (1 default; environment PSGUI_CULL overrides; takes effect at the next
 * set_tree): skip a primitive, or a whole operator subtree, when no point of the wave lies
 * in the world box outside which its field is exactly +0 (bounds through the node
 * matrices, none below warps) -- results are bit-identical either way. */
#define PSGUI_OPT_CULL          2
#define PSGUI_JIT_NONE          0    /* interpreter (no compile requested)               */
#define PSGUI_JIT_PENDING       1    /* compiling; the interpreter serves                */
#define PSGUI_JIT_ACTIVE        2    /* the tree's kernels serve                         */
#define PSGUI_JIT_FAILED        3    /* compile or load failed; the interpreter serves   */
int  psgpu_gui_set_option(psgpu_gui* g, int option, int value);
/* PSGUI_JIT_* of the current tree (wait != 0: block until its compile has finished). */
int  psgpu_gui_jit_status(psgpu_gui* g, int wait);
/* Compile a tree's kernels without a device (validation, cache warm-up): code-object
 * bytes, or -1 with the compiler log in `log`; on success `log` holds the source. */
long psgpu_gui_jit_compile(const PsGuiPrim* prims, uint32_t ctPrims, const PsGuiOp* ops, uint32_t ctOps,
                           const uint32_t* kids, uint32_t ctKids, const PsGuiMatrix* mtx, uint32_t ctMtx, int cull,
                           char* log, size_t cap);
/* The culling boxes set_tree derives (8 floats per primitive / operator: lo xyz, 0, hi xyz,
 * 0; infinite where no exact bound exists, empty for Null); host only (tests, tools). */
int  psgpu_gui_cull_boxes(const PsGuiPrim* prims, uint32_t ctPrims, const PsGuiOp* ops, uint32_t ctOps,
                          const uint32_t* kids, uint32_t ctKids, const PsGuiMatrix* mtx, uint32_t ctMtx,
                          float* primBoxes, float* opBoxes);

#ifdef __cplusplus
} /* extern "C" */
static_assert(sizeof(PsGuiPrim) == 128, "PsGuiPrim size");
static_assert(sizeof(PsGuiOp) == 80, "PsGuiOp size");
static_assert(sizeof(PsGuiInfo) == 56, "PsGuiInfo size");
#else
_Static_assert(sizeof(PsGuiPrim) == 128, "PsGuiPrim size");
_Static_assert(sizeof(PsGuiOp) == 80, "PsGuiOp size");
_Static_assert(sizeof(PsGuiInfo) == 56, "PsGuiInfo size");
#endif

#endif /* PARSIP_GPU_GUI_H */
