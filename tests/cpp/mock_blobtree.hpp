// Test double of the ParsipHaptics BlobTree API that include/parsip_gpu_blobtree.hpp binds
// (Parsip100/PS_BlobTree/include): the same class names and accessors the reference
// SimdPoly::linearizeBlobTree calls (PS_HighPerformanceRender.cpp:42-364), holding values
// read from a tree file written by tests/test_cpp_simdpoly.py.  Not the BlobTree library:
// no field functions, no octree construction; boxes and backward matrices come from the
// Python mirror (parsip_amd/blobtree.py).
#pragma once
#include <cstddef>
#include <cstring>
#include <vector>

namespace PS {
namespace BLOBTREE {

struct vec3f { float x, y, z; };
struct vec4f { float x, y, z, w; };
struct COctree { vec3f lower, upper; };
struct CMaterial { vec4f diffused; };
struct CInterval { float left, right; };
enum MajorAxices { xAxis = 0, yAxis = 1, zAxis = 2 };

struct CMatrix {  // row-major 4x4 (PS_MATRIX: getRow copies row r)
    float e[16];
    bool identity;
    bool isIdentity() const { return identity; }
    void getRow(float* row, int r) const { std::memcpy(row, &e[4 * r], 16); }
};
struct CAffineTransformation {
    CMatrix back;
    CMatrix getBackwardMatrix() const { return back; }
};

class CBlobNode {
public:
    virtual ~CBlobNode() {}
    int type = 0;
    std::vector<CBlobNode*> kids;
    COctree octree{};
    CMaterial material{};
    CAffineTransformation transform{};
    float res[4] = {0, 0, 0, 0};
    int id = -1;

    int getNodeType() { return type; }
    int getID() const { return id; }
    bool isOperator() { return type >= 14; }  // bntOpUnion and up (_constSettings.h:32)
    size_t countChildren() const { return kids.size(); }
    CBlobNode* getChild(size_t i) { return i < kids.size() ? kids[i] : nullptr; }
    COctree getOctree() { return octree; }
    CMaterial getMaterial() const { return material; }
    CAffineTransformation& getTransform() { return transform; }
};

class CSkeleton {
public:
    virtual ~CSkeleton() {}
    vec3f a{}, b{}, c{};
    float r = 0.0f, h = 0.0f;
};
class CSkeletonPoint : public CSkeleton {
public:
    vec3f getPosition() const { return a; }
};
class CSkeletonLine : public CSkeleton {
public:
    vec3f getStartPosition() const { return a; }
    vec3f getEndPosition() const { return b; }
};
class CSkeletonRing : public CSkeleton {
public:
    vec3f getPosition() const { return a; }
    vec3f getDirection() const { return b; }
    float getRadius() const { return r; }
};
class CSkeletonDisc : public CSkeletonRing {};
class CSkeletonCylinder : public CSkeleton {
public:
    vec3f getPosition() const { return a; }
    vec3f getDirection() const { return b; }
    float getRadius() const { return r; }
    float getHeight() const { return h; }
};
class CSkeletonCube : public CSkeleton {
public:
    vec3f getPosition() const { return a; }
    float getSide() const { return r; }
};
class CSkeletonTriangle : public CSkeleton {
public:
    vec3f getTriangleCorner(int i) const { return i == 0 ? a : (i == 1 ? b : c); }
};

class CSkeletonPrimitive : public CBlobNode {
public:
    CSkeleton* skeleton = nullptr;
    ~CSkeletonPrimitive() override { delete skeleton; }
    CSkeleton* getSkeleton() { return skeleton; }
};

class CQuadricPoint : public CBlobNode {  // not a skeletal primitive (CompactBlobTree.cpp:369-377)
public:
    vec3f pos{};
    float radius = 0.0f, scale = 0.0f;
    vec3f getPosition() const { return pos; }
    float getFieldRadius() const { return radius; }
    float getFieldScale() const { return scale; }
};

class CInstance : public CBlobNode {  // CInstance.h:11-82
public:
    CBlobNode* origin = nullptr;
    CBlobNode* getOriginalNode() const { return origin; }
};

class CPcm : public CBlobNode {
public:
    float getPropagateLeft() const { return res[0]; }
    float getPropagateRight() const { return res[1]; }
    float getAlphaLeft() const { return res[2]; }
    float getAlphaRight() const { return res[3]; }
};
class CRicciBlend : public CBlobNode {
public:
    float getN() const { return res[0]; }
};
class CWarpTwist : public CBlobNode {
public:
    float getWarpFactor() const { return res[0]; }
    MajorAxices getMajorAxis() const { return (MajorAxices)(int)res[1]; }
};
class CWarpTaper : public CBlobNode {
public:
    float getWarpFactor() const { return res[0]; }
    MajorAxices getAxisAlong() const { return (MajorAxices)(int)res[1]; }
    MajorAxices getAxisTaper() const { return (MajorAxices)(int)res[2]; }
};
class CWarpBend : public CBlobNode {
public:
    float getBendRate() const { return res[0]; }
    float getBendCenter() const { return res[1]; }
    CInterval getBendRegion() const { return CInterval{res[2], res[3]}; }
};
class CWarpShear : public CBlobNode {
public:
    float getWarpFactor() const { return res[0]; }
    MajorAxices getAxisAlong() const { return (MajorAxices)(int)res[1]; }
    MajorAxices getAxisDependent() const { return (MajorAxices)(int)res[2]; }
};

}  // namespace BLOBTREE
}  // namespace PS
