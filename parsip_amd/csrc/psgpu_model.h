// psgpu_model.h — device-side image of a linearised BlobTree (host + device).
//
// The reference walks the op tree per SIMD call with an explicit stack
// (FieldComputer::fieldValue, PS_Polygonizer.cpp:1184-1376).  On CDNA4 every
// wavefront walks the same tree, so the host flattens the walk once per model into
// a short wave-uniform program (read with scalar loads) and the per-lane state is
// reduced to a resume pc (op-box pruning) plus a small value stack in LDS.
//
//   ENTER  op, skipTo, out   depth>3 op-box test (PS_Polygonizer.cpp:1228-1252);
//                            lanes whose 4-lane group is outside resume at skipTo
//                            with field 0 in slot `out`.
//   PRIM   prim, out         computePrimitiveField (:934-1179) into slot `out`.
//   OP     op, type, l, r    binary combine (:1282-1338) into slot `out`.
//   SUMPRIM prim             no-op trees: running sum of all prims (:1356-1368).
//
// The program order is the reference's processing order (post-order, right child
// first, :1344-1352), which also fixes the "stale outField" semantics of op types
// that have no case in the reference switch.
#pragma once
#ifdef __HIPCC_RTC__
// hiprtc (run-time specialised kernels, psgpu_jit.cpp): no system headers
typedef unsigned char uint8_t;
typedef signed char int8_t;
typedef unsigned short uint16_t;
typedef unsigned int uint32_t;
typedef int int32_t;
typedef unsigned long long uint64_t;
typedef long long int64_t;
#else
#include <stdint.h>
#include <hip/hip_runtime.h>
#endif

namespace psgpu {

// Node type codes of the hot path (PS_Polygonizer.h:84-91; same as PsNodeType).
#define PSGPU_T_CYLINDER 0
#define PSGPU_T_DISC 1
#define PSGPU_T_LINE 2
#define PSGPU_T_POINT 3
#define PSGPU_T_RING 4
#define PSGPU_T_CUBE 6
#define PSGPU_T_TRIANGLE 7
#define PSGPU_T_UNION 14
#define PSGPU_T_INTERSECT 15
#define PSGPU_T_DIF 16
#define PSGPU_T_SMOOTHDIF 17
#define PSGPU_T_BLEND 18
#define PSGPU_T_RICCI 19

// Marching-cubes tables in device memory (generated on the host, psgpu_host.cpp),
// packed so a cell's whole row is one 64-bit word (4 bits per edge id):
//   row[c]   the triangle row g_triTableCache[c] (<= 15 entries)
//   order[c] the row's distinct edges in first-occurrence order (<= 12)
//   cross[c] 12-bit mask of sign-changing edges (== the row's edge set)
//   ntri[c]  triangles in the row
//   own[b]   12-bit mask of edges a cell owns, b = (i==0)<<2 | (j==0)<<1 | (k==0)
//   edge     per edge: corner1 (3 bits) | axis << 3, 5 bits per edge
//   crossNtri[c] cross[c] | ntri[c] << 16 (pass 1's one lookup per cell)
// k_mpu reads them from global memory (the 5.9 KB stay in every CU's L1 / L2).
struct CubeTablesDev {
    uint64_t row[256];
    uint64_t order[256];
    uint16_t cross[256];
    uint8_t ntri[256];
    uint16_t own[8];
    uint64_t edge;
    uint8_t pad[8];
    uint32_t crossNtri[256];
};

enum InstrKind : uint8_t { kEnter = 0, kPrim = 1, kOp = 2, kSumPrim = 3 };

struct Instr {           // 16 B, one s_load_dwordx4
    uint8_t kind;
    uint8_t type;        // OP: op type (PS_Polygonizer.h enum)
    uint8_t out;         // value slot written
    uint8_t lslot;       // OP: slot of left child value
    uint8_t rslot;       // OP: slot of right child value
    uint8_t childKind;   // OP: bit1 left is op, bit0 right is op
    uint8_t L, R;        // OP: child indices (prim or op ids)
    uint16_t idx;        // ENTER/OP: op id; PRIM/SUMPRIM: prim id
    uint16_t skipTo;     // ENTER: pc after the op's OP instruction
    uint32_t pad;
};
static_assert(sizeof(Instr) == 16, "Instr size");

struct DevOp {           // 32 B
    float lo[3];
    float hi[3];
    float resY;          // RicciBlend exponent (SOABlobOps::resY)
    uint32_t type;
};
static_assert(sizeof(DevOp) == 32, "DevOp size");

struct DevPrim {         // 128 B
    float pos[3];
    float dir[3];
    float res[3];
    float col[3];
    uint32_t type;
    uint32_t hasMatrix;  // idxMatrix != 0
    uint32_t cullable;   // bit 0: exact culling bound valid; 1: unbounded line; 2: axis clearance
    float cullRadius;    // skeleton-to-surface slack of the bound (cube: half diagonal)
    float mat[12];       // SOABlobPrimMatrices row-major 3x4 (12-float stride)
    float pad[4];
};
static_assert(sizeof(DevPrim) == 128, "DevPrim size");

constexpr int kMaxInstr = 512;
constexpr int kMaxSlots = 64;

// Culling skeleton of a primitive: the segment A + t*U, t in [tmin, tmax] ([0,1]; any t
// for the unbounded Line), whose distance minus `radius` bounds the primitive's distance
// from below; one branch-free formula for every slot: radius = +inf never culls (not
// eligible, or past ctPrims), -inf always culls (Triangle: field exactly 0).
struct CullSeg {         // 48 B: three 16-B loads per lane
    float a[3];
    float u[3];
    float invUU;         // 1 / |U|^2, 0 for a point
    float radius;
    float tmin, tmax;
    float axisClear;     // the box must keep this distance from the segment's line (Cylinder: its
                         // rounded-negative sqrt is NaN on the axis); -inf: no condition
    float pad;
};
static_assert(sizeof(CullSeg) == 48, "CullSeg size");

struct DevModel {
    uint32_t nInstr;
    uint32_t nSlots;
    uint32_t ctPrims;
    uint32_t ctOps;
    uint32_t boundable;  // 1: field bounds over a box are valid (see prim_bound, psgpu_device.h)
    uint32_t pad[3];
    Instr instr[kMaxInstr];
    DevOp ops[128];
    DevPrim prims[128];
    CullSeg cull[128];
    float zeroCol[128][4];  // colour of op i when every field below it is +0 (see host)
};

// Compact-mesh work records written by the MPU kernel.
// A vertex record in two arrays, so that each kernel moves only what it uses: k_mpu writes
// the key (8 B), k_vertex reads it and writes the root (8 B), k_finish reads both and
// recomputes the position from them with k_vertex's own expressions (vertex_root).
struct VertexKey {       // 8 B: MPU slot in the range, vid | edge key << 16
    uint32_t w;
    uint32_t vidKey;     // vid | key << 16, key = sx | sy<<3 | sz<<6 | axis<<9
};
struct VertexPos {       // 8 B (k_vertex): the linear root's scale on its bracketing segment
    float scale;         // (0.5 - fa) / (fb - fa)
    uint32_t iv;         // the segment [sample iv - 1, sample iv] of the edge's 4 samples (1..3)
};
// Triangle record, 8 B.  An MPU has at most 1,715 triangles and 1,344 edges (11-bit local
// ids); the record sits in queue shard w & 63 of its MPU slot w, so the slot needs only
// w >> 6 (20 bits: ranges of up to 2^26 MPUs, checked by psgpu_polygonize).
struct TriRec {
    uint32_t a;          // tlocal | (v2 >> 10) << 11 | (w >> 6) << 12
    uint32_t b;          // v0 | v1 << 11 | (v2 & 1023) << 22
};
constexpr uint32_t kMaxRangeMpus = 1u << 26;

// Device-side scalars of one polygonization.
// Work records are appended to kShards independent queues so that no single counter
// takes one returning atomic per MPU (a single word saturates at about 88 atomics/us
// on MI355X: MI355X_MICROARCH.md 'dequeue').
constexpr int kShards = 64;
constexpr uint32_t kScanItems = 2048;   // offsets scan: counts per 256-thread block per chunk
constexpr uint32_t kScanMaxBlocks = 256;
struct ShardCtr {           // one 128-B line per shard: atomics on one line serialise
    uint32_t p;             // S1 survivors appended (k_front: shards 0-7 are its 8 sub-queues)
    uint32_t v;             // vertex records appended
    uint32_t t;             // triangle records appended
    uint32_t s;             // surface MPUs (>= 1 triangle)
    uint32_t b;             // S1 survivors proven empty by field bounds (not queued)
    uint32_t s1Done;        // k_front, shards 0-7: S1 blocks of sub-queue k that published all entries
    uint32_t pad[26];
};
struct DevCounters {
    int32_t firstOverflow;   // min global MPU id with > 512 V or T (INT32_MAX: none)
    uint32_t error;          // protocol errors (bit 0: offsets-scan look-back timeout, bit 1: k_surface's
                             // wait for the scan timed out)
    uint32_t scanDone;       // k_surface: offsets-scan blocks finished (released) in this run
    uint32_t surfaceErr;     // host copy only: 2 once a k_surface wave's scan wait timed out (plain
                             // stores of one value, so no read-modify-write over PCIe); zeroed by
                             // k_precheck, never copied from the device counters by k_surface
    uint32_t epoch;          // run sequence number: the previous run's last kernel sets it to its own
                             // + 1 when it resets this set; k_front tags its queue entries with it + 1
    uint32_t pad[27];
    ShardCtr shard[kShards];
};

#ifndef PSGPU_MPU_WAVES
#define PSGPU_MPU_WAVES 1  // waves per S1 survivor in k_mpu (1, 2 or 4): each walks 8 / W of the
                           // 8 x-slices of the S2 cache and takes every W-th batch of records,
                           // so a heavy MPU's critical path is ~1/W of one wave doing it all.
                           // Host and device must agree (build.py and the JIT pass the same value).
                           // C3 ms/step on one box: W=1 0.0624, W=2 0.0669, W=4 0.0722.
#endif
constexpr int kMpuWaves = PSGPU_MPU_WAVES;
constexpr int kMpusPerBlock = 4 / kMpuWaves;  // k_mpu blocks are 4 waves
constexpr int kNumStampKernels = 4;  // k_precheck, k_mpu, k_vertex, k_finish
constexpr int kSpanLanes = 64;       // {min start, max end} pairs per kernel per run (PSGPU_OPT_SPANS)

// Kernel arguments of one polygonization (one struct, passed by value).
struct Params {
    const DevModel* __restrict__ model;
    const CubeTablesDev* __restrict__ tables;
    float cs;           // cellsize
    float side;         // cellsize * 7.0f (MPU side)
    float lo[3];        // scene bboxLo
    uint32_t dims[3];   // MPU lattice
    uint32_t divMagic[2];  // floor((2^32 - 1) / d) for d = dims[2], dims[1] * dims[2] (mpu_origin)
    uint32_t mpuBegin;
    uint32_t mpuCount;
    uint32_t cull;      // exact per-wave primitive culling enabled
    uint32_t preBlocks;     // k_precheck blocks (4 waves, one 2x2x2 brick of MPUs per wave)
    uint32_t brickI0;       // first brick row (x) touching the MPU range
    uint32_t brickDims[3];  // bricks of the range along x, y, z
    uint32_t brickStride;   // wave W takes brick (W * brickStride) mod bricks (coprime: a
                            // permutation that spreads the surface's heavy bricks over the CUs)
    uint32_t* pq;           // kShards queues of pShardCap S1 survivors (global MPU ids)
    uint64_t* pqMask;       // per queue entry: the MPU box's culling mask (2 words, by k_precheck)
    uint16_t* pqOct;        // per queue entry: octants proven all outside (bits 0-7) / inside (8-15)
    uint32_t pShardCap;     // 8 * ceil(precheck waves / kShards): cannot overflow
    uint32_t* fqReady;      // k_front: per queue entry, the run's tag once the entry is published
    uint32_t fqCap;         // k_front: entries per sub-queue (8 sub-queues at pq + k * fqCap)
    uint32_t mpuBlocks;     // k_mpu grid (4 waves per block, kMpusPerBlock queued survivors per block)
    uint64_t* counts;       // mpuCount: V | T << 32 per MPU of the range (0 if S1 failed)
    uint8_t* passed;        // mpuCount: 1 if the MPU passed S1 (PsMpuStats::passedPrecheck)
    uint32_t bound;         // k_precheck proves S1 survivors empty by field bounds
    uint64_t* mpuMasks;     // 2 * mpuCount: culling mask of each queued MPU's box + delta (k_precheck)
    uint64_t* offs;         // mpuCount + 1: exclusive scan of counts
    uint64_t* scanStatus;   // offsets-scan look-back words of this run (zeroed by the previous run)
    uint64_t* scanStatusNext;
    uint32_t scanBlocks;    // offsets-scan blocks (the first blocks of k_vertex)
    uint32_t scanChunks;    // kScanItems chunks per scan block
    VertexKey* vk;          // kShards queues of vShardCap vertex records (keys ...
    VertexPos* vp;          // ... and roots, same indexing)
    uint32_t vShardCap;
    TriRec* tq;             // kShards queues of tShardCap records
    uint32_t tShardCap;
    float* pos;             // vCap vertices
    float* nrm;
    float* col;
    uint32_t* tris;         // tCap triangles
    uint32_t vCap, tCap;
    DevCounters* ctr;       // this run's counters (two sets alternate between runs)
    DevCounters* ctrNext;   // the next run's, reset by k_finish
    DevCounters* hostCtr;   // host-mapped copy written by k_finish
    uint32_t* totals;       // 8 words written by k_finish: MPUs, V, T, passed S1, surface MPUs,
                            // S2 MPUs, first overflow MPU, error (the parts' count exchange)
    uint64_t* stamps;       // per-wave timeline (PSGPU_OPT_STAMPS) or null: kNumStampKernels x
    uint32_t stampCap;      // stampCap records {start, end, item | hw id << 32} (s_memrealtime)
    uint64_t* spans;        // PSGPU_OPT_SPANS: this run's slot, per kernel {first wave start, last
                            // wave end} (atomic min / max of s_memrealtime), or null
    uint64_t* mpuTicks;     // PSGPU_OPT_MPU_TICKS (MPUSTATS): 4 words per MPU of the range -- its S1
                            // wave's start and end, its S2 wave's end (0: not queued), hw ids of the
                            // S1 | S2 waves << 32 (s_memrealtime) -- or null
    uint32_t slotsPerLane;  // value slots (x4 floats in colour mode)
    uint32_t debug;         // ablation switches for profiling (0 in production)
};

}  // namespace psgpu
