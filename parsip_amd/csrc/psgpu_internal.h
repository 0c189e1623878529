// psgpu_internal.h — the device context shared by the library's host sources
// (psgpu_host.cpp: one context, psgpu_group.cpp: contexts over several devices and the
// multi-process count exchange).  Not part of the C-ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <memory>
#include <string>
#include <vector>

#include "../../include/parsip_gpu.h"
#include "psgpu_jit.h"
#include "psgpu_model.h"
#include "psgpu_pool.h"

namespace psgpu {
constexpr int kNumKernels = 4;
}  // namespace psgpu

namespace psgpu {
constexpr int kExportPieces = 16;  // at most, in the blocking export (psgpu_host.cpp export_stage)
constexpr size_t kExportPieceBytes = 1u << 20;  // its target piece size

}  // namespace psgpu

struct psgpu_ctx {
    using JitKernels = psgpu::JitKernels;
    using JitFuture = psgpu::JitFuture;
    using DevModel = psgpu::DevModel;
    using Params = psgpu::Params;
    using DevCounters = psgpu::DevCounters;
    using VertexKey = psgpu::VertexKey;
    using VertexPos = psgpu::VertexPos;
    using TriRec = psgpu::TriRec;
    using CubeTablesDev = psgpu::CubeTablesDev;
    static constexpr int kNumKernels = psgpu::kNumKernels;
    int device = 0;
    uint64_t serial = 0;  // process-unique id: this context's PrintThreadResults entry
    bool countThreads = true;  // finished runs add to that entry (off for a group's planning runs)
    int numCUs = 256;
    hipStream_t stream = nullptr;
    PsSoaBlobPrims primsHost;  // bbox + counts of the current model
    DevModel model{};
    DevModel* dModel = nullptr;
    CubeTablesDev* dTables = nullptr;
    int useJit = 1;
    int jitAsync = 1;                  // set_model returns while hiprtc compiles (interpreter meanwhile)
    std::shared_ptr<JitKernels> jit;   // specialised kernels of the current model
    JitFuture jitFut;                  // the current model's compile, while jitPending
    bool jitPending = false;
    std::string jitError;
    // this run enqueued while no other run of the process was pending on the device (a
    // blocking caller): the layout defaults pick the shorter-span (latency) layouts
    bool alone = false;
    // ... or while 4 or more other contexts have runs pending on it: no in-kernel waits then
    bool crowded = false;
    // PSGPU_OPT_JIT 3 (tiered): once the model has stayed unchanged for tierRuns runs, its
    // baked kernels compile on a host thread and replace the structure kernels (kept in jit1)
    int tier = 0;                      // what `jit` holds: 0 none, 1 structure, 2 baked kernels
    int tierRuns = 16;
    int staticRuns = 0;                // runs of the current model on the structure kernels
    JitFuture tier2Fut;                // the baked compile, while tier2Pending
    bool tier2Pending = false;
    bool tier2Failed = false;          // the baked compile failed: stay on tier 1 for this model
    std::shared_ptr<JitKernels> jit1;  // the structure kernels while tier 2 serves
    std::vector<JitFuture> retired;    // baked compiles of models since replaced (destroy waits)
    bool haveModel = false;
    int cull = 1;
    int debug = 0;
    int vertexBlocksPerCU = 16;  // persistent k_vertex / k_finish grids (256-thread blocks)
    int finishBlocksPerCU = 8;
    int finishQuad = 2;  // PSGPU_OPT_FINISH_QUAD: 0 one lane, 1 a quad, 3 a pair of lanes per vertex, 2 by the last run's vertex count
    int treeSplit = 0;   // PSGPU_OPT_TREE_SPLIT: 1 k_precheck / k_mpu walk the root's two subtrees in two waves
    bool splittable = false;  // the model's walk splits at the root (jit_splittable)
    int fusedSurface = 2;     // PSGPU_OPT_FUSED_SURFACE: k_vertex + k_finish in one launch (use_surface)
    bool runSurface = false;  // the last enqueued run took k_surface
    int front = 2;            // PSGPU_OPT_FRONT: k_precheck + k_mpu in one launch (use_front)
    bool runFront = false;    // the last enqueued run took k_front
    bool runSplit = false;    // ... and the tree-split kernels
    uint32_t lastSubMax = 0;  // the largest k_front sub-queue of the last finished run (0: none)
    uint32_t* fqReady = nullptr;  // k_front: per queue entry, the tag of the run that published it
    size_t capFq = 0;
    bool surfaceOff = false;  // while finish re-runs a run whose in-kernel wait gave up: the separate kernels
    uint32_t splitMaxQueued = 1024;  // PSGPU_OPT_SPLIT_MAX_QUEUED: tree split 2 applies up to this many S2 MPUs
                                     // (psgpu_create: 4 per CU; C3's 1/8 shares queue ~800, 1/4 ~1,600)
    uint32_t runMpb = 0;      // k_mpu MPUs per block of the last enqueued run
    int gridFit = 1;          // k_vertex / k_finish grids sized from the last run's vertices, capped
                              // at the persistent grids (PSGPU_GRID_FIT=0: the persistent grids;
                              // C4 1/8 shares -5 %, full grids neutral: profiles/r05_grid_fit_ab2.txt)
    int mpuMarginDiv = 4;     // k_mpu grid: last run's queued MPUs + 1/this (re-run if short)
    int vertexWide = 2;  // PSGPU_OPT_VERTEX_WIDE: 0 a quad, 1 one lane per vertex, 2 by the last run's vertex count
    uint32_t lastV = 0;  // vertices of the last finished run (0: none yet)
    int timing = 0;
    // geometry of the last run
    float cs = 0.0f;
    uint32_t dims[3] = {0, 0, 0};
    uint32_t mpuBegin = 0, mpuCount = 0;
    hipStream_t runStream = nullptr;
    bool pending = false;
    bool haveResult = false;
    // device buffers
    size_t capLb = 0, capList = 0, capCounts = 0, capOff = 0, capVk = 0, capVp = 0, capTq = 0, capV = 0, capT = 0;
    uint32_t* pq = nullptr;         // sharded S1 survivor queues
    uint64_t* pqMask = nullptr;     // 2 words per queue entry (culling mask of the MPU box)
    uint16_t* pqOct = nullptr;      // per queue entry: octant proofs (Params::pqOct)
    size_t capPqOct = 0;
    size_t capPqMask = 0;
    uint32_t pShardCap = 0;
    uint32_t lastQueued = 0;        // S1 survivors queued for S2 in the last finished run
    bool haveQueued = false;        // lastQueued describes the current range and lattice
    float lastCs = 0.0f;            // the cell size of the last enqueued run
    uint32_t runMpuBlocks = 0;      // k_mpu grid of the last enqueued run
    uint64_t* scanStatus = nullptr; // 2 x kScanMaxBlocks look-back words (alternating runs)
    uint32_t parity = 0;            // which counter / status set the next run uses
    // runs launched since the counter sets last started at epoch 0 = the next run's epoch
    // (DevCounters::epoch; k_front tags its queue entries epoch + 1, which must never wrap to 0)
    uint64_t epochRuns = 0;
    uint64_t* counts = nullptr;
    uint8_t* passed = nullptr;      // per MPU: passed S1
    size_t capPassed = 0;
    int bound = 1;                  // prove S1 survivors empty by field bounds in k_precheck
    uint64_t* mpuMasks = nullptr;
    size_t capMasks = 0;
    uint64_t* offs = nullptr;
    VertexKey* vk = nullptr;
    VertexPos* vp = nullptr;
    TriRec* tq = nullptr;
    float* pos = nullptr;
    float* nrm = nullptr;
    float* col = nullptr;
    uint32_t* tris = nullptr;
    DevCounters* ctr = nullptr;         // two sets, alternating runs
    uint32_t* totals = nullptr;         // 8 words of the last run's totals (k_finish), for RCCL,
    uint32_t* emptyTotals = nullptr;    // then 8 words of an empty run's (totals + 8)
    uint64_t* stamps = nullptr;         // per-wave timeline (PSGPU_OPT_STAMPS), 4 x stampCap x 3 words
    uint32_t stampCap = 0;
    uint64_t* spans = nullptr;          // per-run kernel spans (PSGPU_OPT_SPANS): spanCap x 4 x 2 words
    uint32_t spanCap = 0, spanNext = 0;
    int mpuTicksOpt = 0;                // PSGPU_OPT_MPU_TICKS: runs record per-MPU ticks (MPUSTATS)
    uint64_t* mpuTicks = nullptr;       // 4 words per MPU of the range (Params::mpuTicks)
    size_t capTicks = 0;
    bool runTicks = false;              // the last enqueued run recorded them
    uint64_t* clockProbe = nullptr;     // pinned, mapped: one device clock reading (k_clock_probe)
    DevCounters* hostCtr = nullptr;     // pinned, mapped: written by k_finish
    DevCounters* hostCtrDev = nullptr;  // its device address
    unsigned char* hostStage = nullptr;  // pinned staging for the blocking PolyMPUs export
    size_t hostStageCap = 0;
    hipEvent_t exportEv[2] = {};         // the export's metadata, then its packing kernel
    uint32_t exportEpoch = 0;            // the blocking export's flag value (k_export_pack), never 0
    std::unique_ptr<psgpu::ScatterPool> scatterPool;  // the export's scatter threads, made on first use
    uint32_t vcap = 1u << 20, tcap = 1u << 21;               // compact mesh capacity
    uint32_t vShardCap = 1u << 15, tShardCap = 1u << 16;      // work-queue capacity per shard
    hipEvent_t ev[kNumKernels + 1] = {};
    int useGraph = 0;  // replay repeated launch sequences from a hipGraph (measured slower on ROCm 7.2)
    struct GraphSlot {
        hipGraphExec_t exec = nullptr;
        JitKernels* jit = nullptr;
        Params key{};
        uint32_t shape[6] = {0, 0, 0, 0, 0, 0};
    } graphs[2];
    float lastMs[kNumKernels] = {};
    PsMeshInfo info{};
    // high-water marks of finished runs: the next run's buffers are sized from them
    // (an animation whose mesh grows frame to frame does not pay a synchronous re-run)
    uint32_t seenV = 0, seenT = 0, seenShardV = 0, seenShardT = 0;
};


namespace psgpu {
// HIP error -> library return code (prints the failing call).
int hip_fail(hipError_t e, const char* what);
// Make the context's device current on the calling thread.
int set_device(psgpu_ctx* c);
// The blocking export of a finished run in two steps (psgpu_host.cpp): enqueue the copies of
// the compact mesh (mesh), the S1 flags and (stats) the per-MPU counts into the context's
// pinned staging buffer, then wait and scatter into PolyMPUs / PsMpuStats.
struct ExportStage {
    bool mesh = false, stats = false;
    size_t V = 0, T = 0, N = 0;
    size_t oOffs = 0, oPos = 0, oNrm = 0, oCol = 0, oTris = 0, oPass = 0, oCnt = 0;
    // the mesh, packed as `pieces` MPU ranges (pos | nrm | col | 16-bit triangle corners of
    // each, psgpu_launch.h PackSrc) at oMesh, piece k complete when its packBlocks flags at
    // oFlags + 4 k packBlocks equal epoch: the scatter of one piece overlaps the
    // transfer of the next.  oFlags = 0 in every call: the flag words hold nothing else
    int pieces = 0;
    size_t oMesh = 0, meshBytes = 0, oFlags = 0;
    uint32_t epoch = 0, packBlocks = 0;
};
// `after`: an event the packing kernel waits for (the previous part's packing on the same
// device, so the parts' pieces cross the link in range order)
int export_stage(psgpu_ctx* c, bool mesh, bool stats, ExportStage* st, hipEvent_t after = nullptr);
int export_scatter(psgpu_ctx* c, const ExportStage& st, PsMPU* mpus, PsMpuStats* stats, const int64_t* trace = nullptr);
bool export_trace_on();
inline int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
// One staged export's scatter into PolyMPUs, split so that a group's parts go in one pass of
// the thread pool (scatter_jobs): prepare (after the metadata), task per thread, finish.
struct ScatterJob {
    psgpu_ctx* c = nullptr;
    const ExportStage* S = nullptr;
    PsMPU* mpus = nullptr;
    const uint64_t* off = nullptr;
    const uint8_t* passed = nullptr;
    const unsigned char* mesh = nullptr;
    const uint32_t* flags = nullptr;
    float side = 0.0f;
    bool active = false;
    std::atomic<bool> failed{false};
    uint32_t pm[kExportPieces + 1] = {};
    size_t pbase[kExportPieces] = {}, pv0[kExportPieces] = {}, pt0[kExportPieces] = {}, pnv[kExportPieces] = {};
    int prepare(psgpu_ctx* c, const ExportStage& st, PsMPU* mpus);
    std::atomic<int> ready{0};        // pieces known to be in (-1: the packing kernel failed)
    // PSGPU_EXPORT_TRACE: steady-clock ns when the first scatter task started, when each piece
    // was seen in (export_blocking prints the call's phases to stderr)
    bool trace = false;
    std::atomic<int64_t> tFirstTask{0};
    int64_t tPiece[kExportPieces] = {};
    std::atomic<bool> polling{false};  // a thread is reading the flags
    uint32_t pollBlock = 0;            // the poller's place in the current piece's flags (under `polling`)
    bool wait_piece(int k);
    bool range(uint32_t lb, uint32_t le, int* have);
    void task(unsigned k, unsigned nth);
    int finish(PsMpuStats* stats);
};
int scatter_jobs(psgpu_ctx* c, ScatterJob* jobs, size_t n);
}  // namespace psgpu

#define PSGPU_CHECK(expr)                                           \
    do {                                                            \
        hipError_t _e = (expr);                                     \
        if (_e != hipSuccess) return psgpu::hip_fail(_e, #expr);    \
    } while (0)
