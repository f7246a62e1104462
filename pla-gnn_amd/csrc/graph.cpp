// Host-side graph construction for the plagnn C-ABI.
//
// Replaces what DGL does below code/utils.py:44-45 (dgl.graph((start, end), N) then
// dgl.add_self_loop) and at the first update_all (code/model.py:20): the COO edge list
// (self-loops already appended by the caller with edge ids E..E+N-1) becomes the
// in-CSR that DGL's SpMMCmpCsr walks, each destination row listing its in-edges in
// ascending edge id. Also builds the transposed (out-)CSR used by the deterministic
// max backward, and the per-row work schedule the device kernels consume.
#include <algorithm>
#include <array>
#include <cstdlib>
#include <new>
#include <vector>

#include "common.hpp"

namespace pg {

char* error_buffer() {
  static thread_local char buf[512];
  return buf;
}

int set_error(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(error_buffer(), 512, fmt, ap);
  va_end(ap);
  return code;
}

}  // namespace pg

extern "C" {

const char* pg_last_error_string(void) { return pg::error_buffer(); }

int pg_version(void) { return 13; }

int pg_csr_from_coo(const int64_t* src, const int64_t* dst, int64_t nnz, int64_t n_src,
                    int64_t n_dst, int32_t* ptr, int32_t* col, int32_t* eid) {
  if (nnz < 0 || n_src < 0 || n_dst < 0)
    return pg::set_error(PG_ERR_INVALID, "pg_csr_from_coo: negative size");
  if (nnz > INT32_MAX || n_src > INT32_MAX || n_dst > INT32_MAX)
    return pg::set_error(PG_ERR_UNSUPPORTED, "pg_csr_from_coo: graph exceeds int32 ids");
  if (!ptr || (nnz > 0 && (!src || !dst || !col)))
    return pg::set_error(PG_ERR_INVALID, "pg_csr_from_coo: NULL buffer");
  // validate ids first so no partial output is left on error
  for (int64_t e = 0; e < nnz; ++e) {
    if (src[e] < 0 || src[e] >= n_src || dst[e] < 0 || dst[e] >= n_dst)
      return pg::set_error(PG_ERR_INVALID,
                           "pg_csr_from_coo: edge %lld (%lld -> %lld) out of range [0,%lld)x[0,%lld)",
                           (long long)e, (long long)src[e], (long long)dst[e], (long long)n_src,
                           (long long)n_dst);
  }
  // counting sort by dst; scanning edges in id order keeps each row stable
  std::fill(ptr, ptr + n_dst + 1, 0);
  for (int64_t e = 0; e < nnz; ++e) ptr[dst[e] + 1]++;
  for (int64_t v = 0; v < n_dst; ++v) ptr[v + 1] += ptr[v];
  std::vector<int32_t> cursor;
  try {
    cursor.assign(ptr, ptr + n_dst);
  } catch (const std::bad_alloc&) {
    return pg::set_error(PG_ERR_HOST, "pg_csr_from_coo: out of host memory");
  }
  for (int64_t e = 0; e < nnz; ++e) {
    const int32_t k = cursor[dst[e]]++;
    col[k] = (int32_t)src[e];
    if (eid) eid[k] = (int32_t)e;
  }
  return pg::ok();
}

int pg_csr_transpose(const int32_t* ptr, const int32_t* col, int64_t n_rows, int64_t n_cols,
                     int64_t nnz, int32_t* tptr, int32_t* tcol, int32_t* tslot, int32_t* tpos) {
  if (n_rows < 0 || n_cols < 0 || nnz < 0)
    return pg::set_error(PG_ERR_INVALID, "pg_csr_transpose: negative size");
  if (!ptr || !tptr || (nnz > 0 && (!col || !tcol)))
    return pg::set_error(PG_ERR_INVALID, "pg_csr_transpose: NULL buffer");
  if (ptr[0] != 0 || ptr[n_rows] != nnz)
    return pg::set_error(PG_ERR_INVALID, "pg_csr_transpose: ptr does not span nnz");
  for (int64_t k = 0; k < nnz; ++k)
    if (col[k] < 0 || col[k] >= n_cols)
      return pg::set_error(PG_ERR_INVALID, "pg_csr_transpose: col[%lld]=%d out of range",
                           (long long)k, col[k]);
  std::fill(tptr, tptr + n_cols + 1, 0);
  for (int64_t k = 0; k < nnz; ++k) tptr[col[k] + 1]++;
  for (int64_t c = 0; c < n_cols; ++c) tptr[c + 1] += tptr[c];
  std::vector<int32_t> cursor;
  try {
    cursor.assign(tptr, tptr + n_cols);
  } catch (const std::bad_alloc&) {
    return pg::set_error(PG_ERR_HOST, "pg_csr_transpose: out of host memory");
  }
  // rows visited ascending -> every transposed row lists its entries in ascending row id
  for (int64_t r = 0; r < n_rows; ++r) {
    for (int32_t k = ptr[r]; k < ptr[r + 1]; ++k) {
      const int32_t t = cursor[col[k]]++;
      tcol[t] = (int32_t)r;
      if (tslot) tslot[t] = k;
      if (tpos) tpos[t] = k - ptr[r];
    }
  }
  return pg::ok();
}

int pg_schedule_count(const int32_t* ptr, int64_t n_rows, int32_t chunk, int64_t* n_items,
                      int64_t* n_merges, int64_t* n_slots, int32_t* max_deg) {
  if (!ptr || n_rows < 0 || chunk <= 0)
    return pg::set_error(PG_ERR_INVALID, "pg_schedule_count: bad arguments");
  int64_t items = 0, merges = 0, slots = 0;
  int32_t md = 0;
  for (int64_t r = 0; r < n_rows; ++r) {
    const int32_t d = ptr[r + 1] - ptr[r];
    if (d < 0) return pg::set_error(PG_ERR_INVALID, "pg_schedule_count: ptr not monotone");
    md = std::max(md, d);
    if (d <= chunk) {
      items += 1;
    } else {
      const int64_t n = (d + (int64_t)chunk - 1) / chunk;
      items += n;
      merges += 1;
      slots += n;
    }
  }
  if (n_items) *n_items = items;
  if (n_merges) *n_merges = merges;
  if (n_slots) *n_slots = slots;
  if (max_deg) *max_deg = md;
  return pg::ok();
}

int pg_schedule_build(const int32_t* ptr, int64_t n_rows, int32_t chunk, int32_t* items,
                      int32_t* merges) {
  if (!ptr || n_rows < 0 || chunk <= 0 || (n_rows > 0 && !items))
    return pg::set_error(PG_ERR_INVALID, "pg_schedule_build: bad arguments");
  // Emit items, then order them longest-first (counting sort on length, stable in row
  // order) so the heaviest pieces start first and the tail of the launch is short.
  std::vector<int32_t> raw;
  try {
    raw.reserve((size_t)n_rows * 4);
  } catch (const std::bad_alloc&) {
    return pg::set_error(PG_ERR_HOST, "pg_schedule_build: out of host memory");
  }
  int32_t slot = 0;
  int64_t m = 0;
  for (int64_t r = 0; r < n_rows; ++r) {
    const int32_t b = ptr[r], e = ptr[r + 1];
    const int32_t d = e - b;
    if (d <= chunk) {
      raw.insert(raw.end(), {(int32_t)r, b, e, -1});
    } else {
      const int32_t n = (d + chunk - 1) / chunk;
      if (merges) {
        merges[4 * m + 0] = (int32_t)r;
        merges[4 * m + 1] = slot;
        merges[4 * m + 2] = n;
        merges[4 * m + 3] = 0;
      }
      ++m;
      for (int32_t i = 0; i < n; ++i) {
        const int32_t k0 = b + i * chunk;
        const int32_t k1 = std::min(e, k0 + chunk);
        raw.insert(raw.end(), {(int32_t)r, k0, k1, slot + i});
      }
      slot += n;
    }
  }
  // split rows longest first too (the sliced max forward takes each as a whole workgroup,
  // in this order); a stable sort keeps equal lengths in row order
  if (merges && m > 1) {
    std::vector<std::array<int32_t, 4>> ms((size_t)m);
    for (int64_t i = 0; i < m; ++i) std::copy(merges + 4 * i, merges + 4 * i + 4, ms[(size_t)i].begin());
    std::stable_sort(ms.begin(), ms.end(), [](const auto& a, const auto& b) { return a[2] > b[2]; });
    for (int64_t i = 0; i < m; ++i) std::copy(ms[(size_t)i].begin(), ms[(size_t)i].end(), merges + 4 * i);
  }
  const int64_t n_items = (int64_t)raw.size() / 4;
  std::vector<int64_t> bucket((size_t)chunk + 2, 0);
  for (int64_t i = 0; i < n_items; ++i) bucket[chunk - (raw[4 * i + 2] - raw[4 * i + 1]) + 1]++;
  for (size_t i = 1; i < bucket.size(); ++i) bucket[i] += bucket[i - 1];
  for (int64_t i = 0; i < n_items; ++i) {
    const int32_t len = raw[4 * i + 2] - raw[4 * i + 1];
    const int64_t at = bucket[chunk - len]++;
    std::copy(&raw[4 * i], &raw[4 * i] + 4, items + 4 * at);
  }
  return pg::ok();
}

}  // extern "C"
