/* psoracle.h — TEST INFRASTRUCTURE ONLY (see psoracle.c header). */
#ifndef PSORACLE_H
#define PSORACLE_H
#include <stdint.h>
#include "../include/parsip_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct PsModelRef {
    const PsSoaBlobPrims* prims;
    const PsSoaPrimMatrices* mats;
    const PsSoaBlobOps* ops;
} PsModelRef;

typedef struct psor_result psor_result;

void psor_tritable(int32_t out[256 * 16]);
float psor_prim_field1(const PsModelRef* m, uint32_t idx, float x, float y, float z);
void psor_field_value(const PsModelRef* m, const float* x4, const float* y4, const float* z4, float* out4);
void psor_field_value_and_color(const PsModelRef* m, const float* x4, const float* y4, const float* z4,
                                float* f4, float* cx4, float* cy4, float* cz4);
uint32_t psor_count_mpus(float cs, const float lo[3], const float hi[3]);
int psor_polygonize(float cellsize, const PsModelRef* m, uint32_t mpuBegin, uint32_t mpuEnd, int nthreads,
                    int keepMesh, psor_result** out);
void psor_result_info(const psor_result* r, uint32_t* ctMPUs, uint32_t* ctV, uint32_t* ctT);
void psor_result_copy(const psor_result* r, uint32_t* stats5, float* pos, float* nrm, float* col, uint16_t* tri);
void psor_result_free(psor_result* r);
void psor_work_counts(uint64_t out[5 * 64]);
int psor_prepare_bboxes(PsSoaBlobPrims* P, const PsSoaBoxMatrices* BM, PsSoaBlobOps* O);

#ifdef __cplusplus
}
#endif
#endif
