// psgpu_group.cpp — one grid over several devices (C-ABI, include/parsip_gpu.h).
//
// The reference's Polygonize is ONE blocking call that fans the whole MPU list over every
// core (tbb::parallel_for over CMPUProcessor, PS_Polygonizer.cpp:379-382).  The MI355X
// equivalent fans one MPU lattice over the node's GPUs:
//
//   psgpu_group_*   one process, one context per device: contiguous MPU ranges of
//                   near-equal cost (psgpu_split_costs over psgpu_mpu_costs of a planning
//                   run), launched on every device's stream at once; the count exchange is
//                   a host read of each part's totals; psgpu_group_gather assembles the
//                   parts on one device with peer copies over xGMI (hipMemcpyPeerAsync) and
//                   a rebase kernel, or psgpu_group_download_mesh to the host.
//   psgpu_comm_*    one process per GPU (torchrun / MPI launchers): each rank owns a range
//                   of the same split (computed identically on every rank) and the parts'
//                   totals are exchanged with one RCCL all-gather of 8 words per rank on
//                   the context's stream, right after its k_finish (stream-ordered, no
//                   host round trip inside a frame).
//
// MPUs are independent (each evaluates its own 8^3 corners, faces included), so the
// concatenation of the parts in range order IS the single-device mesh: no halo, no
// data-path collective.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <vector>

#include "psgpu_internal.h"
#include "psgpu_launch.h"

using namespace psgpu;

struct psgpu_group {
    std::vector<psgpu_ctx*> parts;
    std::vector<uint32_t> bounds;   // parts + 1 global MPU ids
    int balance = 1;                // PSGPU_GROUP_BALANCE_*
    uint32_t minPartMpus = 0;       // PSGPU_GROUP_OPT_MIN_PART_MPUS
    bool planned = false;           // bounds are a cost split of the current lattice
    float planCs = 0.0f;
    PsVec3f planLo{}, planHi{};
    bool pending = false;
    bool haveResult = false;
    std::vector<PsMeshInfo> info;   // per part, after finish
    std::vector<uint32_t> vBase, tBase;
    PsMeshInfo total{};
    // gathered mesh (psgpu_group_gather) on one part's device
    int gatherPart = -1;
    hipStream_t gatherStream = nullptr;
    float *gPos = nullptr, *gNrm = nullptr, *gCol = nullptr;
    uint32_t* gTris = nullptr;
    uint64_t* gOffs = nullptr;
    size_t gCapV = 0, gCapT = 0, gCapM = 0;
    // one rank's parts summed for the RCCL exchange (psgpu_comm_exchange_group)
    std::vector<hipEvent_t> done;
    uint32_t* sumTotals = nullptr;
};

namespace {

void free_gather(psgpu_group* g) {
    if (g->gatherPart < 0) return;
    (void)hipSetDevice(g->parts[g->gatherPart]->device);
    if (g->gatherStream) (void)hipStreamSynchronize(g->gatherStream);
    void* bufs[] = {g->gPos, g->gNrm, g->gCol, g->gTris, g->gOffs};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    if (g->gatherStream) (void)hipStreamDestroy(g->gatherStream);
    g->gPos = g->gNrm = g->gCol = nullptr;
    g->gTris = nullptr;
    g->gOffs = nullptr;
    g->gatherStream = nullptr;
    g->gCapV = g->gCapT = g->gCapM = 0;
    g->gatherPart = -1;
}

uint32_t lattice_total(psgpu_group* g, float cs) {
    uint32_t dims[3] = {0, 0, 0};
    if (psgpu_mpu_dims(cs, &g->parts[0]->primsHost, dims) != PSGPU_RET_SUCCESS) return 0;
    const uint64_t t = (uint64_t)dims[0] * dims[1] * dims[2];
    return t > 0xffffffffull ? 0u : (uint32_t)t;
}

bool same_lattice(const psgpu_group* g, float cs) {
    const PsSoaBlobPrims& P = g->parts[0]->primsHost;
    return g->planned && g->planCs == cs && !memcmp(&g->planLo, &P.bboxLo, sizeof(PsVec3f)) &&
           !memcmp(&g->planHi, &P.bboxHi, sizeof(PsVec3f));
}

// MPUs per planning run: below the per-run limit (PSGPU_PLAN_CHUNK_MPUS lowers it, so tests
// exercise the chunked plan on small lattices)
uint32_t plan_chunk_mpus() {
    uint32_t chunk = kMaxRangeMpus - 1u;
    if (const char* v = getenv("PSGPU_PLAN_CHUNK_MPUS")) {
        const long x = strtol(v, nullptr, 10);
        if (x > 0 && (uint64_t)x < chunk) chunk = (uint32_t)x;
    }
    return chunk;
}

// Parts that get a range: all, or with PSGPU_GROUP_OPT_MIN_PART_MPUS the first
// total / minPartMpus of them (at least one); the rest get empty ranges at the end.
uint32_t active_parts(const psgpu_group* g, uint32_t total) {
    const uint32_t n = (uint32_t)g->parts.size();
    if (!g->minPartMpus) return n;
    return std::max(1u, std::min(n, total / g->minPartMpus));
}

void even_split(psgpu_group* g, uint32_t total) {
    const uint32_t n = (uint32_t)g->parts.size(), a = active_parts(g, total);
    g->bounds.assign(n + 1, total);
    for (uint32_t k = 0; k < a; ++k) g->bounds[k] = (uint32_t)((uint64_t)total * k / a);
}

// Cost split of the lattice from a planning run of the whole grid on part 0 (one
// polygonization per chunk of fewer than kMaxRangeMpus MPUs, the most one run takes;
// results are exact, so every caller that plans the same model and lattice gets the same
// split).
int plan(psgpu_group* g, float cs, uint32_t total) {
    const uint32_t n = (uint32_t)g->parts.size(), a = active_parts(g, total);
    g->bounds.assign(n + 1, total);
    g->bounds[0] = 0;
    if (a > 1 && total > 0) {
        std::vector<uint32_t> costs(total);
        // planning runs are not the caller's polygonizations: PrintThreadResults skips them
        g->parts[0]->countThreads = false;
        for (uint32_t b = 0; b < total;) {
            const uint32_t e = (uint32_t)std::min<uint64_t>(total, (uint64_t)b + plan_chunk_mpus());
            int rc = psgpu_polygonize(g->parts[0], cs, b, e, nullptr);
            if (rc == PSGPU_RET_SUCCESS) rc = psgpu_mpu_costs(g->parts[0], costs.data() + b);
            if (rc != PSGPU_RET_SUCCESS) {
                g->parts[0]->countThreads = true;
                return rc;
            }
            b = e;
        }
        g->parts[0]->countThreads = true;
        const int rc = psgpu_split_costs(costs.data(), total, a, 0, g->bounds.data());
        if (rc != PSGPU_RET_SUCCESS) return rc;
    }
    const PsSoaBlobPrims& P = g->parts[0]->primsHost;
    g->planLo = P.bboxLo;
    g->planHi = P.bboxHi;
    g->planCs = cs;
    g->planned = true;
    return PSGPU_RET_SUCCESS;
}

// Re-split from the costs of the run just finished (PSGPU_GROUP_BALANCE_EVERY_RUN).
int replan_from_last(psgpu_group* g) {
    const uint32_t n = (uint32_t)g->parts.size();
    const uint32_t begin = g->bounds[0], total = g->bounds[n] - g->bounds[0];
    std::vector<uint32_t> costs(total);
    for (uint32_t p = 0; p < n; ++p) {
        if (g->bounds[p + 1] == g->bounds[p]) continue;
        const int rc = psgpu_mpu_costs(g->parts[p], costs.data() + (g->bounds[p] - begin));
        if (rc != PSGPU_RET_SUCCESS) return rc;
    }
    const uint32_t a = active_parts(g, total);
    std::fill(g->bounds.begin(), g->bounds.end(), begin + total);
    return psgpu_split_costs(costs.data(), total, a, begin, g->bounds.data());
}

}  // namespace

extern "C" {

int psgpu_group_create(const int* devices, int nParts, psgpu_group** out) {
    if (!out || nParts <= 0 || nParts > 64) return PSGPU_RET_PARAM_ERROR;
    *out = nullptr;
    const int ndev = psgpu_device_count();
    if (ndev <= 0) return PSGPU_RET_DEVICE_ERROR;
    psgpu_group* g = new psgpu_group();
    for (int p = 0; p < nParts; ++p) {
        const int d = devices ? devices[p] : p;
        psgpu_ctx* c = nullptr;
        const int rc = (d >= 0 && d < ndev) ? psgpu_create(d, &c) : PSGPU_RET_DEVICE_ERROR;
        if (rc != PSGPU_RET_SUCCESS) {
            psgpu_group_destroy(g);
            return rc;
        }
        g->parts.push_back(c);
    }
    // direct peer access between the parts' devices (xGMI) for the gather; a pair
    // without it still copies (staged by the runtime)
    for (psgpu_ctx* a : g->parts)
        for (psgpu_ctx* b : g->parts) {
            if (a->device == b->device) continue;
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, a->device, b->device) == hipSuccess && can) {
                (void)hipSetDevice(a->device);
                const hipError_t e = hipDeviceEnablePeerAccess(b->device, 0);
                if (e != hipSuccess) (void)hipGetLastError();  // already enabled is fine
            }
        }
    *out = g;
    return PSGPU_RET_SUCCESS;
}

void psgpu_group_destroy(psgpu_group* g) {
    if (!g) return;
    free_gather(g);
    if (!g->parts.empty()) (void)hipSetDevice(g->parts[0]->device);
    for (hipEvent_t e : g->done)
        if (e) (void)hipEventDestroy(e);
    if (g->sumTotals) (void)hipFree(g->sumTotals);
    for (psgpu_ctx* c : g->parts) psgpu_destroy(c);
    delete g;
}

int psgpu_group_size(psgpu_group* g) { return g ? (int)g->parts.size() : 0; }

psgpu_ctx* psgpu_group_context(psgpu_group* g, int part) {
    return (g && part >= 0 && part < (int)g->parts.size()) ? g->parts[part] : nullptr;
}

int psgpu_group_set_option(psgpu_group* g, int option, int64_t value) {
    if (!g) return PSGPU_RET_PARAM_ERROR;
    if (option == PSGPU_GROUP_OPT_BALANCE) {
        if (value < 0 || value > 3) return PSGPU_RET_PARAM_ERROR;
        g->balance = (int)value;
        g->planned = false;
        return PSGPU_RET_SUCCESS;
    }
    if (option == PSGPU_GROUP_OPT_MIN_PART_MPUS) {
        if (value < 0 || value > 0xffffffffll) return PSGPU_RET_PARAM_ERROR;
        g->minPartMpus = (uint32_t)value;
        g->planned = false;
        g->bounds.clear();  // re-split at the next polygonize
        return PSGPU_RET_SUCCESS;
    }
    for (psgpu_ctx* c : g->parts) {
        const int rc = psgpu_set_option(c, option, value);
        if (rc != PSGPU_RET_SUCCESS) return rc;
    }
    return PSGPU_RET_SUCCESS;
}

int psgpu_group_set_model(psgpu_group* g, const PsSoaBlobPrims* prims, const PsSoaPrimMatrices* mats,
                          const PsSoaBlobOps* ops) {
    if (!g) return PSGPU_RET_PARAM_ERROR;
    // one hiprtc job serves every part (jit_request dedups by source); each device loads it
    for (psgpu_ctx* c : g->parts) {
        const int rc = psgpu_set_model(c, prims, mats, ops);
        if (rc != PSGPU_RET_SUCCESS) return rc;
    }
    g->haveResult = false;
    return PSGPU_RET_SUCCESS;
}

int psgpu_group_jit_wait(psgpu_group* g) {
    if (!g) return 0;
    int all = 1;
    for (psgpu_ctx* c : g->parts) all &= psgpu_jit_wait(c);
    return all;
}

int psgpu_group_set_split(psgpu_group* g, const uint32_t* bounds) {
    if (!g || !bounds) return PSGPU_RET_PARAM_ERROR;
    const size_t n = g->parts.size();
    for (size_t k = 0; k < n; ++k)
        if (bounds[k] > bounds[k + 1]) return PSGPU_RET_PARAM_ERROR;
    g->bounds.assign(bounds, bounds + n + 1);
    g->balance = PSGPU_GROUP_BALANCE_FIXED;
    g->planned = false;
    return PSGPU_RET_SUCCESS;
}

int psgpu_group_get_split(psgpu_group* g, uint32_t* bounds) {
    if (!g || !bounds || g->bounds.size() != g->parts.size() + 1) return PSGPU_RET_PARAM_ERROR;
    std::copy(g->bounds.begin(), g->bounds.end(), bounds);
    return PSGPU_RET_SUCCESS;
}

int psgpu_group_polygonize(psgpu_group* g, float cellsize) {
    if (!g || !g->parts[0]->haveModel || !(cellsize > 0.0f)) return PSGPU_RET_PARAM_ERROR;
    const uint32_t total = lattice_total(g, cellsize);
    const size_t n = g->parts.size();
    const bool replan = g->balance == PSGPU_GROUP_BALANCE_PLAN &&
                        (!same_lattice(g, cellsize) || g->bounds.size() != n + 1 || g->bounds[n] != total);
    if (g->pending && (replan || g->balance == PSGPU_GROUP_BALANCE_EVERY_RUN)) {
        // the split depends on the previous run: finish it first (else runs queue up per
        // part stream, each context double-buffers its counters)
        PsMeshInfo tmp;
        const int rc = psgpu_group_finish(g, &tmp, nullptr);
        if (rc != PSGPU_RET_SUCCESS) return rc;
    }
    if (g->balance == PSGPU_GROUP_BALANCE_FIXED) {
        if (g->bounds.size() != n + 1) even_split(g, total);
    } else if (g->balance == PSGPU_GROUP_BALANCE_EVEN) {
        even_split(g, total);
    } else if (replan || (g->balance == PSGPU_GROUP_BALANCE_EVERY_RUN && !same_lattice(g, cellsize))) {
        const int rc = plan(g, cellsize, total);
        if (rc != PSGPU_RET_SUCCESS) return rc;
    }
    // every device gets its range at once: the launches are asynchronous, per device stream
    for (size_t p = 0; p < n; ++p) {
        const int rc = psgpu_polygonize(g->parts[p], cellsize, g->bounds[p], g->bounds[p + 1], nullptr);
        if (rc != PSGPU_RET_SUCCESS) return rc;
    }
    g->pending = true;
    g->haveResult = false;
    return PSGPU_RET_SUCCESS;
}

int psgpu_group_finish(psgpu_group* g, PsMeshInfo* totalOut, PsGroupPart* partsOut) {
    if (!g) return PSGPU_RET_PARAM_ERROR;
    const size_t n = g->parts.size();
    if (g->pending) {
        g->pending = false;
        g->info.assign(n, PsMeshInfo{});
        for (size_t p = 0; p < n; ++p) {
            const int rc = psgpu_finish(g->parts[p], &g->info[p]);
            if (rc != PSGPU_RET_SUCCESS) return rc;
        }
        // the count exchange: each part's place in the global index space
        g->vBase.assign(n, 0);
        g->tBase.assign(n, 0);
        PsMeshInfo& T = g->total;
        memset(&T, 0, sizeof(T));
        T.firstOverflowMPU = -1;
        uint64_t v = 0, t = 0;
        for (size_t p = 0; p < n; ++p) {
            const PsMeshInfo& I = g->info[p];
            g->vBase[p] = (uint32_t)v;
            g->tBase[p] = (uint32_t)t;
            v += I.ctVertices;
            t += I.ctTriangles;
            T.ctMPUs += I.ctMPUs;
            T.ctPassedPrecheck += I.ctPassedPrecheck;
            T.ctSurfaceMPUs += I.ctSurfaceMPUs;
            T.ctLaneEvals += I.ctLaneEvals;
            T.ctFieldMPUs += I.ctFieldMPUs;
            T.launchFlags |= I.launchFlags;  // any part's
            if (I.firstOverflowMPU >= 0 && T.firstOverflowMPU < 0) T.firstOverflowMPU = I.firstOverflowMPU;
        }
        if (v > 0xffffffffull || t > 0xffffffffull) return PSGPU_RET_NOT_ENOUGH_MEM;
        T.ctVertices = (uint32_t)v;
        T.ctTriangles = (uint32_t)t;
        g->haveResult = true;
        if (g->balance == PSGPU_GROUP_BALANCE_EVERY_RUN && n > 1) {
            const int rc = replan_from_last(g);
            if (rc != PSGPU_RET_SUCCESS) return rc;
        }
    }
    if (!g->haveResult) return PSGPU_RET_PARAM_ERROR;
    if (totalOut) *totalOut = g->total;
    if (partsOut) {
        for (size_t p = 0; p < n; ++p) {
            PsGroupPart& P = partsOut[p];
            P.device = g->parts[p]->device;
            P.mpuBegin = g->parts[p]->mpuBegin;
            P.mpuEnd = g->parts[p]->mpuBegin + g->parts[p]->mpuCount;
            P.vertexBase = g->vBase[p];
            P.triangleBase = g->tBase[p];
            P.info = g->info[p];
        }
    }
    return PSGPU_RET_SUCCESS;
}

// The whole mesh on the host, exactly as one device would produce it: part p's
// vertices at its vertex base, its triangle ids and MPU offsets rebased.
int psgpu_group_download_mesh(psgpu_group* g, float* pos, float* nrm, float* col, uint32_t* tris,
                              uint64_t* mpuOffsets) {
    PsMeshInfo T;
    int rc = psgpu_group_finish(g, &T, nullptr);
    if (rc != PSGPU_RET_SUCCESS) return rc;
    const size_t n = g->parts.size();
    uint64_t mBase = 0;
    std::vector<uint64_t> offs;
    for (size_t p = 0; p < n; ++p) {
        const PsMeshInfo& I = g->info[p];
        const size_t vb = g->vBase[p], tb = g->tBase[p];
        offs.assign((size_t)I.ctMPUs + 1, 0);
        rc = psgpu_download_mesh(g->parts[p], pos ? pos + vb * 3 : nullptr, nrm ? nrm + vb * 3 : nullptr,
                                 col ? col + vb * 3 : nullptr, tris ? tris + tb * 3 : nullptr, offs.data());
        if (rc != PSGPU_RET_SUCCESS) return rc;
        if (tris)
            for (size_t i = tb * 3; i < (tb + I.ctTriangles) * 3; ++i) tris[i] += (uint32_t)vb;
        if (mpuOffsets) {
            const uint64_t add = (uint64_t)vb | ((uint64_t)tb << 32);
            for (size_t i = 0; i <= I.ctMPUs; ++i) mpuOffsets[mBase + i] = offs[i] + add;
        }
        mBase += I.ctMPUs;
    }
    if (mpuOffsets && mBase == 0) mpuOffsets[0] = 0;
    return PSGPU_RET_SUCCESS;
}

// The whole mesh in HBM of one part's device: peer copies of every part (xGMI), then the
// rebase kernel per part.  The returned pointers stay valid until the next gather.
int psgpu_group_gather(psgpu_group* g, int dstPart, PsMeshDevice* out) {
    if (!g || !out || dstPart < 0 || dstPart >= (int)g->parts.size()) return PSGPU_RET_PARAM_ERROR;
    PsMeshInfo T;
    int rc = psgpu_group_finish(g, &T, nullptr);
    if (rc != PSGPU_RET_SUCCESS) return rc;
    if (g->gatherPart != dstPart) free_gather(g);
    psgpu_ctx* dst = g->parts[dstPart];
    PSGPU_CHECK(hipSetDevice(dst->device));
    if (!g->gatherStream) PSGPU_CHECK(hipStreamCreateWithFlags(&g->gatherStream, hipStreamNonBlocking));
    g->gatherPart = dstPart;
    const size_t V = std::max<size_t>(T.ctVertices, 1), Tn = std::max<size_t>(T.ctTriangles, 1),
                 M = (size_t)T.ctMPUs + 1;
    auto grow = [](auto*& ptr, size_t& cap, size_t need, size_t elt) -> hipError_t {
        if (need <= cap && ptr) return hipSuccess;
        if (ptr) (void)hipFree(ptr);
        ptr = nullptr;
        hipError_t e = hipMalloc(reinterpret_cast<void**>(&ptr), need * elt);
        cap = e == hipSuccess ? need : 0;
        return e;
    };
    size_t capV2 = g->gCapV, capV3 = g->gCapV;
    PSGPU_CHECK(grow(g->gPos, g->gCapV, V, 12));
    PSGPU_CHECK(grow(g->gNrm, capV2, V, 12));
    PSGPU_CHECK(grow(g->gCol, capV3, V, 12));
    PSGPU_CHECK(grow(g->gTris, g->gCapT, Tn, 12));
    PSGPU_CHECK(grow(g->gOffs, g->gCapM, M, 8));
    hipStream_t s = g->gatherStream;
    uint64_t mBase = 0;
    for (size_t p = 0; p < g->parts.size(); ++p) {
        psgpu_ctx* c = g->parts[p];
        const PsMeshInfo& I = g->info[p];
        PsMeshDevice src;
        rc = psgpu_mesh_device(c, &src);
        if (rc != PSGPU_RET_SUCCESS) return rc;
        PSGPU_CHECK(hipSetDevice(dst->device));
        const size_t vb = g->vBase[p], tb = g->tBase[p];
        const int sd = c->device, dd = dst->device;
        if (I.ctVertices) {
            PSGPU_CHECK(hipMemcpyPeerAsync(g->gPos + vb * 3, dd, src.pos, sd, (size_t)I.ctVertices * 12, s));
            PSGPU_CHECK(hipMemcpyPeerAsync(g->gNrm + vb * 3, dd, src.nrm, sd, (size_t)I.ctVertices * 12, s));
            PSGPU_CHECK(hipMemcpyPeerAsync(g->gCol + vb * 3, dd, src.col, sd, (size_t)I.ctVertices * 12, s));
        }
        if (I.ctTriangles)
            PSGPU_CHECK(hipMemcpyPeerAsync(g->gTris + tb * 3, dd, src.tris, sd, (size_t)I.ctTriangles * 12, s));
        if (I.ctMPUs)
            PSGPU_CHECK(hipMemcpyPeerAsync(g->gOffs + mBase, dd, src.mpuOffsets, sd, ((size_t)I.ctMPUs + 1) * 8, s));
        PSGPU_CHECK(launch_rebase(g->gTris + tb * 3, (uint64_t)I.ctTriangles * 3, (uint32_t)vb, g->gOffs + mBase,
                                  I.ctMPUs ? (uint64_t)I.ctMPUs + 1 : 0, (uint64_t)vb | ((uint64_t)tb << 32), s));
        mBase += I.ctMPUs;
    }
    if (mBase == 0) PSGPU_CHECK(hipMemsetAsync(g->gOffs, 0, 8, s));
    PSGPU_CHECK(hipStreamSynchronize(s));
    out->pos = g->gPos;
    out->nrm = g->gNrm;
    out->col = g->gCol;
    out->tris = g->gTris;
    out->mpuOffsets = g->gOffs;
    return PSGPU_RET_SUCCESS;
}

int psgpu_group_export_polympus(psgpu_group* g, PsMPU* mpus, uint32_t capacity, uint32_t* outCt) {
    PsMeshInfo T;
    int rc = psgpu_group_finish(g, &T, nullptr);
    if (rc != PSGPU_RET_SUCCESS) return rc;
    if (outCt) *outCt = T.ctMPUs;
    if (T.ctMPUs > capacity) return PSGPU_RET_MPU_OVERFLOW;
    if (T.firstOverflowMPU >= 0) return PSGPU_RET_MPU_VT_OVERFLOW;
    if (!mpus) return PSGPU_RET_PARAM_ERROR;
    // every part's packing first (each on its own stream)
    std::vector<ExportStage> st(g->parts.size());
    for (size_t p = 0; p < g->parts.size(); ++p) {
        rc = set_device(g->parts[p]);
        // parts on one device share its link: each part's packing waits for the previous
        // part's, so the pieces arrive in range order, as the scatter threads take them
        hipEvent_t after =
            p > 0 && g->parts[p - 1]->device == g->parts[p]->device ? g->parts[p - 1]->exportEv[1] : nullptr;
        if (rc == PSGPU_RET_SUCCESS) rc = export_stage(g->parts[p], true, false, &st[p], after);
        if (rc != PSGPU_RET_SUCCESS) return rc;
    }
    // then one pass of the first part's scatter threads over every part, in range order per
    // thread: the parts' packing kernels share the link, the threads follow them
    std::vector<ScatterJob> jobs(g->parts.size());
    uint32_t at = 0;
    for (size_t p = 0; p < g->parts.size(); ++p) {
        rc = jobs[p].prepare(g->parts[p], st[p], mpus + at);
        if (rc != PSGPU_RET_SUCCESS) return rc;
        at += g->parts[p]->mpuCount;
    }
    rc = scatter_jobs(g->parts[0], jobs.data(), jobs.size());
    for (size_t p = 0; p < g->parts.size() && rc == PSGPU_RET_SUCCESS; ++p) {
        rc = set_device(g->parts[p]);
        if (rc == PSGPU_RET_SUCCESS) rc = jobs[p].finish(nullptr);
    }
    return rc;
}

int psgpu_group_polygonize_mpus(psgpu_group* g, float cellsize, const PsSoaBlobPrims* prims,
                                const PsSoaPrimMatrices* mats, const PsSoaBlobOps* ops, PsMPU* mpus,
                                uint32_t capacity, uint32_t* outCt) {
    if (!g || !prims) return PSGPU_RET_PARAM_ERROR;
    if (prims->ctPrims == 0) return PSGPU_RET_PARAM_ERROR;  // Polygonize :322-323
    int rc = psgpu_group_set_model(g, prims, mats, ops);
    if (rc != PSGPU_RET_SUCCESS) return rc;
    rc = psgpu_group_polygonize(g, cellsize);
    if (rc != PSGPU_RET_SUCCESS) return rc;
    return psgpu_group_export_polympus(g, mpus, capacity, outCt);
}

// ---------------------------------------------------------------------------
// Multi-process form: one rank per GPU, RCCL over xGMI for the count exchange.
struct psgpu_comm {
    ncclComm_t comm = nullptr;
    int nranks = 0, rank = 0, device = 0;
    uint32_t* gathered = nullptr;      // device: nranks x 8 words
    uint32_t* hostGathered = nullptr;  // pinned copy
    uint32_t* flag = nullptr;          // device: the "some rank re-ran" all-reduce word, then a
                                       // constant 2 (a failed rank's contribution, no copy needed)
    uint32_t* hostFlag = nullptr;      // pinned
    bool pending = false;
    bool reexchanged = false;          // the last result needed the second exchange
    psgpu_ctx* ctx = nullptr;          // the context whose run was exchanged
    psgpu_group* group = nullptr;      // or the group whose parts were summed
};

static int nccl_fail(ncclResult_t r, const char* what) {
    if (r == ncclSuccess) return PSGPU_RET_SUCCESS;
    fprintf(stderr, "psgpu: %s failed: %s\n", what, ncclGetErrorString(r));
    return PSGPU_RET_DEVICE_ERROR;
}

int psgpu_comm_unique_id(uint8_t id[PSGPU_COMM_ID_BYTES]) {
    static_assert(sizeof(ncclUniqueId) == PSGPU_COMM_ID_BYTES, "ncclUniqueId size");
    if (!id) return PSGPU_RET_PARAM_ERROR;
    ncclUniqueId u;
    const int rc = nccl_fail(ncclGetUniqueId(&u), "ncclGetUniqueId");
    if (rc == PSGPU_RET_SUCCESS) memcpy(id, &u, sizeof(u));
    return rc;
}

int psgpu_comm_create(psgpu_ctx* ctx, const uint8_t id[PSGPU_COMM_ID_BYTES], int nranks, int rank,
                      psgpu_comm** out) {
    if (!ctx || !id || !out || nranks <= 0 || rank < 0 || rank >= nranks) return PSGPU_RET_PARAM_ERROR;
    *out = nullptr;
    int rc = set_device(ctx);
    if (rc != PSGPU_RET_SUCCESS) return rc;
    psgpu_comm* m = new psgpu_comm();
    m->nranks = nranks;
    m->rank = rank;
    m->device = ctx->device;
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    rc = nccl_fail(ncclCommInitRank(&m->comm, nranks, u, rank), "ncclCommInitRank");
    if (rc == PSGPU_RET_SUCCESS &&
        (hipMalloc(&m->gathered, (size_t)nranks * 8 * sizeof(uint32_t)) != hipSuccess ||
         hipHostMalloc(&m->hostGathered, (size_t)nranks * 8 * sizeof(uint32_t), hipHostMallocDefault) != hipSuccess ||
         hipMalloc(&m->flag, 2 * sizeof(uint32_t)) != hipSuccess ||
         hipHostMalloc(&m->hostFlag, 9 * sizeof(uint32_t), hipHostMallocDefault) != hipSuccess))
        rc = PSGPU_RET_DEVICE_ERROR;
    if (rc == PSGPU_RET_SUCCESS) {
        const uint32_t failWords[2] = {0u, 2u};
        if (hipMemcpy(m->flag, failWords, sizeof(failWords), hipMemcpyHostToDevice) != hipSuccess)
            rc = PSGPU_RET_DEVICE_ERROR;
    }
    if (rc != PSGPU_RET_SUCCESS) {
        psgpu_comm_destroy(m);
        return rc;
    }
    *out = m;
    return PSGPU_RET_SUCCESS;
}

void psgpu_comm_destroy(psgpu_comm* m) {
    if (!m) return;
    (void)hipSetDevice(m->device);
    if (m->comm) (void)ncclCommDestroy(m->comm);
    if (m->gathered) (void)hipFree(m->gathered);
    if (m->hostGathered) (void)hipHostFree(m->hostGathered);
    if (m->flag) (void)hipFree(m->flag);
    if (m->hostFlag) (void)hipHostFree(m->hostFlag);
    delete m;
}

// Enqueue the exchange of the context's last polygonization (its k_finish totals) on the
// context's stream: ncclAllGather of 8 words per rank (psgpu_comm_result copies them to the host).
int psgpu_comm_exchange(psgpu_comm* m, psgpu_ctx* ctx) {
    if (!m || !m->comm || !ctx || ctx->device != m->device) return PSGPU_RET_PARAM_ERROR;
    int rc = set_device(ctx);
    if (rc != PSGPU_RET_SUCCESS) return rc;
    hipStream_t s = ctx->runStream ? ctx->runStream : ctx->stream;
    rc = nccl_fail(ncclAllGather(ctx->totals, m->gathered, 8, ncclUint32, m->comm, s), "ncclAllGather");
    if (rc != PSGPU_RET_SUCCESS) return rc;
    m->pending = true;
    m->ctx = ctx;
    m->group = nullptr;
    return PSGPU_RET_SUCCESS;
}

// The same for a rank whose range runs as a group of parts on its one device (several
// streams): part 0's stream waits for the others' last launches, sums their totals and
// all-gathers the sum.
int psgpu_comm_exchange_group(psgpu_comm* m, psgpu_group* g) {
    if (!m || !m->comm || !g || g->parts.empty() || g->parts.size() > 16) return PSGPU_RET_PARAM_ERROR;
    for (psgpu_ctx* c : g->parts)
        if (c->device != m->device) return PSGPU_RET_PARAM_ERROR;
    psgpu_ctx* c0 = g->parts[0];
    int rc = set_device(c0);
    if (rc != PSGPU_RET_SUCCESS) return rc;
    if (g->done.size() != g->parts.size()) {
        for (hipEvent_t e : g->done)
            if (e) (void)hipEventDestroy(e);
        g->done.assign(g->parts.size(), nullptr);
        for (hipEvent_t& e : g->done) PSGPU_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    if (!g->sumTotals) PSGPU_CHECK(hipMalloc(&g->sumTotals, 8 * sizeof(uint32_t)));
    hipStream_t s0 = c0->runStream ? c0->runStream : c0->stream;
    TotalsParts tp{};
    tp.n = (int)g->parts.size();
    for (size_t k = 0; k < g->parts.size(); ++k) {
        psgpu_ctx* c = g->parts[k];
        tp.p[k] = c->totals;
        hipStream_t sk = c->runStream ? c->runStream : c->stream;
        if (sk != s0) {
            PSGPU_CHECK(hipEventRecord(g->done[k], sk));
            PSGPU_CHECK(hipStreamWaitEvent(s0, g->done[k], 0));
        }
    }
    PSGPU_CHECK(launch_sum_totals(tp, g->sumTotals, s0));
    rc = nccl_fail(ncclAllGather(g->sumTotals, m->gathered, 8, ncclUint32, m->comm, s0), "ncclAllGather");
    if (rc != PSGPU_RET_SUCCESS) return rc;
    m->pending = true;
    m->ctx = c0;
    m->group = g;
    return PSGPU_RET_SUCCESS;
}

// After the exchange: every rank's part (MPU range from the gathered counts, bases in
// rank order) and the totals over all ranks.  Finishes the context.  finish() re-runs a
// polygonization whose buffers or k_mpu grid fell short, after its totals were already
// exchanged; whether any rank did so is itself agreed collectively (an all-reduce MAX of a
// flag, on every rank), and then EVERY rank exchanges again -- a collective entered by only
// the ranks that re-ran would block them forever and leave the others with stale counts.
// A rank whose finish fails still enters the all-reduce, with flag 2: then every rank
// returns an error (its own, or PSGPU_RET_DEVICE_ERROR for another rank's failure) and
// none waits for a collective the failed rank will not enter.
// If even that cannot be prepared (the device cannot be made current, or the flag cannot be
// copied to it), the rank still enters the all-reduce, from the constant 2 kept beside the flag
// (no copy needed); should the collective itself fail to enqueue (on this path or on the
// normal one), the communicator is aborted (ncclCommAbort) and unusable from then on --
// psgpu_comm_destroy is all that is left to call.
int psgpu_comm_result(psgpu_comm* m, PsMeshInfo* totalOut, PsGroupPart* partsOut) {
    if (!m || !m->pending || !m->ctx || !m->comm) return PSGPU_RET_PARAM_ERROR;
    psgpu_ctx* c = m->ctx;
    PsMeshInfo mine;
    int local = m->group ? psgpu_group_finish(m->group, &mine, nullptr) : psgpu_finish(c, &mine);
    m->pending = false;
    hipStream_t s = c->runStream ? c->runStream : c->stream;
    auto enter_failed = [&](int rc) {  // this rank's flag 2, so that no other rank waits forever
        if (ncclAllReduce(m->flag + 1, m->flag, 1, ncclUint32, ncclMax, m->comm, s) != ncclSuccess ||
            hipStreamSynchronize(s) != hipSuccess) {
            (void)ncclCommAbort(m->comm);
            m->comm = nullptr;
        }
        return rc;
    };
    if (hipSetDevice(m->device) != hipSuccess) return enter_failed(local != PSGPU_RET_SUCCESS ? local : PSGPU_RET_DEVICE_ERROR);
    const size_t gb = (size_t)m->nranks * 8 * sizeof(uint32_t);
    uint32_t flag = 2u;
    if (local == PSGPU_RET_SUCCESS) {
        // this rank's totals as exchanged vs the totals of its final run (all 8 words: counts,
        // the first overflowing MPU, the error word), both to the host in one wait; the
        // gathered words come to the host only here (not per step: one HIP call less on the
        // host's enqueue path, which bounds small rank shares)
        const uint32_t* finalWords = c->totals;
        if (m->group && m->group->sumTotals) {  // the parts' final totals, summed as exchange_group does
            TotalsParts tp{};
            tp.n = (int)m->group->parts.size();
            for (size_t k = 0; k < m->group->parts.size(); ++k) tp.p[k] = m->group->parts[k]->totals;
            if (launch_sum_totals(tp, m->group->sumTotals, s) != hipSuccess) local = PSGPU_RET_DEVICE_ERROR;
            finalWords = m->group->sumTotals;
        }
        if (local == PSGPU_RET_SUCCESS &&
            (hipMemcpyAsync(m->hostGathered, m->gathered, gb, hipMemcpyDeviceToHost, s) != hipSuccess ||
             hipMemcpyAsync(m->hostFlag + 1, finalWords, 8 * sizeof(uint32_t), hipMemcpyDeviceToHost, s) != hipSuccess ||
             hipStreamSynchronize(s) != hipSuccess))
            local = PSGPU_RET_DEVICE_ERROR;
        if (local == PSGPU_RET_SUCCESS)
            flag = memcmp(m->hostGathered + 8 * m->rank, m->hostFlag + 1, 8 * sizeof(uint32_t)) != 0 ? 1u : 0u;
    }
    *m->hostFlag = flag;
    if (hipMemcpyAsync(m->flag, m->hostFlag, sizeof(uint32_t), hipMemcpyHostToDevice, s) != hipSuccess)
        return enter_failed(local != PSGPU_RET_SUCCESS ? local : PSGPU_RET_DEVICE_ERROR);
    int rc = nccl_fail(ncclAllReduce(m->flag, m->flag, 1, ncclUint32, ncclMax, m->comm, s), "ncclAllReduce");
    if (rc != PSGPU_RET_SUCCESS) {  // the other ranks may be inside the all-reduce: abort it for them
        (void)ncclCommAbort(m->comm);
        m->comm = nullptr;
        return local != PSGPU_RET_SUCCESS ? local : rc;
    }
    PSGPU_CHECK(hipMemcpyAsync(m->hostFlag, m->flag, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    PSGPU_CHECK(hipStreamSynchronize(s));
    if (local != PSGPU_RET_SUCCESS) return local;
    if (*m->hostFlag >= 2u) return PSGPU_RET_DEVICE_ERROR;  // another rank's finish failed
    m->reexchanged = *m->hostFlag != 0u;
    if (m->reexchanged) {  // some rank's totals changed after the exchange: all ranks exchange again
        rc = m->group ? psgpu_comm_exchange_group(m, m->group) : psgpu_comm_exchange(m, c);
        if (rc != PSGPU_RET_SUCCESS) return rc;
        PSGPU_CHECK(hipMemcpyAsync(m->hostGathered, m->gathered, gb, hipMemcpyDeviceToHost, s));
        PSGPU_CHECK(hipStreamSynchronize(s));
    }
    m->pending = false;
    PsMeshInfo T;
    memset(&T, 0, sizeof(T));
    T.firstOverflowMPU = -1;
    uint64_t v = 0, t = 0;
    uint32_t mb = 0;
    for (int r = 0; r < m->nranks; ++r) {
        const uint32_t* w = m->hostGathered + 8 * r;
        if (w[7]) return PSGPU_RET_DEVICE_ERROR;  // a rank's device protocol error
        if (partsOut) {
            PsGroupPart& P = partsOut[r];
            memset(&P, 0, sizeof(P));
            P.device = r == m->rank ? c->device : -1;
            P.mpuBegin = mb;
            P.mpuEnd = mb + w[0];
            P.vertexBase = (uint32_t)v;
            P.triangleBase = (uint32_t)t;
            P.info.ctMPUs = w[0];
            P.info.ctVertices = w[1];
            P.info.ctTriangles = w[2];
            P.info.ctPassedPrecheck = w[3];
            P.info.ctSurfaceMPUs = w[4];
            P.info.ctFieldMPUs = w[5];
            P.info.firstOverflowMPU = w[6] == 0x7fffffffu ? -1 : (int32_t)w[6];
            P.info.ctLaneEvals = 8ull * w[0] + 512ull * w[5] + 8ull * w[1];
        }
        mb += w[0];
        v += w[1];
        t += w[2];
        T.ctMPUs += w[0];
        T.ctPassedPrecheck += w[3];
        T.ctSurfaceMPUs += w[4];
        T.ctFieldMPUs += w[5];
        T.ctLaneEvals += 8ull * w[0] + 512ull * w[5] + 8ull * w[1];
        if (w[6] != 0x7fffffffu && T.firstOverflowMPU < 0) T.firstOverflowMPU = (int32_t)w[6];
    }
    if (v > 0xffffffffull || t > 0xffffffffull) return PSGPU_RET_NOT_ENOUGH_MEM;
    T.ctVertices = (uint32_t)v;
    T.ctTriangles = (uint32_t)t;
    if (totalOut) *totalOut = T;
    return PSGPU_RET_SUCCESS;
}

int psgpu_comm_reexchanged(psgpu_comm* m) { return (m && m->reexchanged) ? 1 : 0; }

}  // extern "C"
