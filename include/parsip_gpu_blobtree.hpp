/*
 * parsip_gpu_blobtree.hpp — SimdPoly for ParsipHaptics' own BlobTree classes.
 *
 * Drop-in for Parsip100/ParsipHaptics/include/PS_HighPerformanceRender.h: include it
 * (after the BlobTree library, Parsip100/PS_BlobTree/include/BlobTreeLibraryAll.h)
 * instead of that header, and the layer that owns a SimdPoly (CLayerManager.h:70,135)
 * keeps calling
 *
 *     SimdPoly poly;
 *     poly.linearizeBlobTree(root);   // PS_HighPerformanceRender.cpp:366-371
 *     poly.run(cellsize);             // :373-376, now on the MI355X
 *     poly.draw(visitor);             // :378-426, the per-MPU arrays handed to GL
 *
 * The node classes named here are the reference's (PS::BLOBTREE, PS_BlobTree/include/):
 * CBlobNode (CBlobTree.h:29), CSkeletonPrimitive (CSkeletonPrimitive.h:24), the skeletons
 * CSkeletonPoint/Line/Ring/Disc/Cylinder/Cube/Triangle, CQuadricPoint, and the operators
 * CPcm, CRicciBlend, CWarpTwist, CWarpTaper, CWarpBend, CWarpShear, CInstance.  It also binds the
 * compat mode (parsip_gpu_gui.hpp) as PS::CParsipOptimizedGpu.
 */
#ifndef PARSIP_GPU_BLOBTREE_HPP
#define PARSIP_GPU_BLOBTREE_HPP

#include "parsip_gpu.hpp"
#include "parsip_gpu_gui.hpp"

struct ParsipBlobTreeApi {
    typedef PS::BLOBTREE::CBlobNode Node;
    typedef PS::BLOBTREE::CSkeletonPrimitive SkeletonPrimitive;
    typedef PS::BLOBTREE::CSkeletonPoint SkeletonPoint;
    typedef PS::BLOBTREE::CSkeletonLine SkeletonLine;
    typedef PS::BLOBTREE::CSkeletonRing SkeletonRing;
    typedef PS::BLOBTREE::CSkeletonDisc SkeletonDisc;
    typedef PS::BLOBTREE::CSkeletonCylinder SkeletonCylinder;
    typedef PS::BLOBTREE::CSkeletonCube SkeletonCube;
    typedef PS::BLOBTREE::CSkeletonTriangle SkeletonTriangle;
    typedef PS::BLOBTREE::CPcm Pcm;
    typedef PS::BLOBTREE::CRicciBlend RicciBlend;
    typedef PS::BLOBTREE::CWarpTwist WarpTwist;
    typedef PS::BLOBTREE::CWarpTaper WarpTaper;
    typedef PS::BLOBTREE::CWarpBend WarpBend;
    typedef PS::BLOBTREE::CWarpShear WarpShear;
    typedef PS::BLOBTREE::CQuadricPoint QuadricPoint;  // compat mode only (parsip_gpu_gui.hpp)
    typedef PS::BLOBTREE::CInstance Instance;          // compat mode only
};

/* class SimdPoly (PS_HighPerformanceRender.h:15-33) on the device. */
typedef psgpu::SimdPolyT<ParsipBlobTreeApi> SimdPoly;

/* The GUI's own polygonizer (CParsipOptimized over a COMPACTBLOBTREE, CPolyParsipOptimized.h:
 * 226-305) on the device: setup takes the BlobTree root (the compact conversion runs inside),
 * the rest keeps the reference's names (run, countMPUs, stats*, drawMesh, exportMesh). */
namespace PS {
typedef psgpu::ParsipOptimizedT<ParsipBlobTreeApi> CParsipOptimizedGpu;
typedef psgpu::CompactTreeT<ParsipBlobTreeApi> COMPACTBLOBTREEGpu;
}  // namespace PS

#endif /* PARSIP_GPU_BLOBTREE_HPP */
