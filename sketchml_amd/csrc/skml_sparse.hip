// skml_sparse.hip -- sparse path (placeholder until the device implementation lands).
#include "skml_sparse.h"

namespace skml {
void sparse_ws_free(SparseWorkspace* w) {
    if (w->buf) (void)hipFree(w->buf);
    w->buf = nullptr;
    w->cap = 0;
}
}  // namespace skml

extern "C" {
static int nyi() { return skml::set_error(SKML_E_STATE, "sparse path not built yet"); }
int skml_sparse_compact_f32(skml_ctx*, const float*, int64_t, int32_t*, float*, int64_t*) { return nyi(); }
int skml_sparse_encode_kv_f32(skml_ctx*, const int32_t*, const float*, int64_t, const skml_params*, skml_sparse**) { return nyi(); }
int skml_sparse_encode_f32(skml_ctx*, const float*, int64_t, const skml_params*, skml_sparse**) { return nyi(); }
int skml_sparse_decode_f32(skml_ctx*, const skml_sparse*, int32_t*, float*) { return nyi(); }
int skml_sparse_nnz(const skml_sparse*, int64_t*) { return nyi(); }
int skml_sparse_quant_info(const skml_sparse*, skml_dense_header*, double*, int32_t) { return nyi(); }
int skml_sparse_group_info(skml_ctx*, const skml_sparse*, int32_t, skml_sparse_group*, int32_t*, uint64_t*, uint64_t*) { return nyi(); }
int skml_sparse_serialize(skml_ctx*, const skml_sparse*, uint8_t*, size_t, size_t*) { return nyi(); }
int skml_sparse_free(skml_sparse*) { return SKML_OK; }
int skml_delta_encode(skml_ctx*, const int32_t*, int64_t, int32_t*, int32_t*, int64_t*, int64_t*, uint64_t*, uint64_t*, int64_t) { return nyi(); }
int skml_delta_decode(skml_ctx*, int64_t, int32_t, int32_t, const uint64_t*, int64_t, const uint64_t*, int64_t, int32_t*) { return nyi(); }
}
