// Shared helpers of the plagnn C-ABI: thread-local error text, argument checks,
// launch-error translation. Included by every translation unit of libplagnn.so.
#pragma once

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "../../include/plagnn.h"

namespace pg {

// Thread-local error string returned by pg_last_error_string().
char* error_buffer();
int set_error(int code, const char* fmt, ...);

inline int ok() {
  error_buffer()[0] = '\0';
  return PG_OK;
}

// Arg-kind helpers
inline bool valid_arg_kind(int k) { return k == PG_ARG_U16 || k == PG_ARG_I32; }
inline size_t arg_bytes(int k) { return k == PG_ARG_U16 ? 2 : 4; }

inline int check_csr(const pg_csr_t* g, const char* who, bool need_sched) {
  if (!g) return set_error(PG_ERR_INVALID, "%s: csr descriptor is NULL", who);
  if (g->n_rows < 0 || g->n_cols < 0 || g->nnz < 0)
    return set_error(PG_ERR_INVALID, "%s: negative csr size", who);
  if (g->n_rows > INT32_MAX || g->n_cols > INT32_MAX || g->nnz > INT32_MAX)
    return set_error(PG_ERR_UNSUPPORTED, "%s: csr larger than int32 ids", who);
  if (!g->ptr) return set_error(PG_ERR_INVALID, "%s: csr ptr is NULL", who);
  if (g->nnz > 0 && !g->col) return set_error(PG_ERR_INVALID, "%s: csr col is NULL", who);
  if (need_sched) {
    if (g->n_rows > 0 && (!g->items || g->n_items <= 0))
      return set_error(PG_ERR_INVALID, "%s: csr has no work schedule", who);
    if (g->n_merges > 0 && !g->merges)
      return set_error(PG_ERR_INVALID, "%s: csr merges missing", who);
  }
  return PG_OK;
}

}  // namespace pg

#define PG_TRY(expr)            \
  do {                          \
    int _rc = (expr);           \
    if (_rc != PG_OK) return _rc; \
  } while (0)
