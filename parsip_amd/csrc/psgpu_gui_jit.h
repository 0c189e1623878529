// psgpu_gui_jit.h -- per-tree compat-mode kernels (hiprtc), see psgpu_gui_jit.cpp.
#pragma once
#include <string>
#include <vector>

#include "../../include/parsip_gpu_gui.h"

namespace psgui {

// HIP source of jit_gui_classify / jit_gui_vertices / jit_gui_probe for one compact tree
// (its structure: node types, kid lists, matrix flags; parameters stay in device memory).
// primBoxes / opBoxes: cull_boxes' output (nullptr: no culling).
std::string jit_source(const PsGuiPrim* P, uint32_t nP, const PsGuiOp* O, uint32_t nO, const uint32_t* K,
                       const float* primBoxes, const float* opBoxes);

// World boxes outside which each primitive's field / operator subtree's value is exactly +0
// (8 floats each: lo xyz, 0, hi xyz, 0; infinite where no exact bound exists).
void cull_boxes(const PsGuiPrim* P, uint32_t nP, const PsGuiOp* O, uint32_t nO, const uint32_t* K,
                const PsGuiMatrix* M, uint32_t nM, std::vector<float>& primBoxes, std::vector<float>& opBoxes);

}  // namespace psgui
