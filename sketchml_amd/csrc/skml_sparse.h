// skml_sparse.h -- sparse-path workspace shared between skml_api.cpp and skml_sparse.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/skml.h"

namespace skml {

struct SparseWorkspace {
    void* buf = nullptr;
    size_t cap = 0;
};
void sparse_ws_free(SparseWorkspace* w);

// accessors into the opaque context (skml_api.cpp)
hipStream_t ctx_stream(skml_ctx* c);
int ctx_device(skml_ctx* c);
SparseWorkspace* ctx_sparse_ws(skml_ctx* c);
int set_error(int code, const char* msg);

}  // namespace skml
