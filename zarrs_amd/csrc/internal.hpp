// Internal accessors shared by the libzgpu translation units (not part of the C ABI).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>

#include "../../include/zgpu.h"
#include "chain.hpp"

namespace zgpu {

// set the calling thread's zgpu_last_error message; returns status
int set_last_error(int status, const std::string &msg);
zgpu_ctx *chain_ctx(const zgpu_chain *c);
// context references (zgpu_ctx::refs): chains, plans and caches hold one each
void ctx_ref(zgpu_ctx *c);
void ctx_unref(zgpu_ctx *c);
const Chain &chain_model(const zgpu_chain *c);
bool chain_validates(const zgpu_chain *c);
int ctx_device(const zgpu_ctx *c);
// the context's caching device allocator (grow-only pools: a steady-state caller performs no
// hipMalloc) and a second stream of its own for copies; both take the context lock
void *ctx_dev_alloc(zgpu_ctx *c, size_t bytes);
void ctx_dev_free(zgpu_ctx *c, void *p);
hipStream_t ctx_copy_stream(zgpu_ctx *c);
// array_read_ops_common.rs:20-109: subset -> one full/partial descriptor per intersecting chunk (C
// order of the chunk grid), lins[k] = descriptor k's linear chunk-grid index. ZGPU_OK, -1 for an empty
// subset, or an error status.
int subset_descs(uint32_t nd, const uint64_t *array_shape, const uint64_t *chunk_shape, const uint64_t *sel_start,
                 const uint64_t *sel_shape, std::vector<zgpu_chunk_desc> &descs, std::vector<uint64_t> &lins);

}  // namespace zgpu
