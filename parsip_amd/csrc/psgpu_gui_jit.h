// psgpu_gui_jit.h -- per-tree compat-mode kernels (hiprtc), see psgpu_gui_jit.cpp.
#pragma once
#include <string>

#include "../../include/parsip_gpu_gui.h"

namespace psgui {

// HIP source of jit_gui_classify / jit_gui_vertices / jit_gui_probe for one compact tree
// (its structure: node types, kid lists, matrix flags; parameters stay in device memory).
std::string jit_source(const PsGuiPrim* P, uint32_t nP, const PsGuiOp* O, uint32_t nO, const uint32_t* K);

}  // namespace psgui
