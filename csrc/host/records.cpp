#include "records.h"

#include <cmath>
#include <cstdlib>

namespace ssa {

UnpackStats unpack_records(const float* packed, int64_t F, int K, int64_t row_stride,
                           const double* meta, Record* out, int64_t cap) {
  UnpackStats st;
  for (int64_t f = 0; f < F; ++f) {
    const float* row = packed + f * row_stride;
    const float raw = row[0];
    int64_t n;
    if (std::isnan(raw)) {
      ++st.pool_lost;
      continue;
    }
    if (raw < 0.f) ++st.overflow;
    n = (int64_t)std::fabs(raw);  // truncation, as numpy's astype(int64) of |count|
    if (n > K) n = K;
    const int64_t fid = (int64_t)meta[3 * f + 0];
    const int32_t stream = (int32_t)(int64_t)meta[3 * f + 1];
    const double ts = meta[3 * f + 2];
    for (int64_t k = 0; k < n && st.records < cap; ++k) {
      const float* r = row + 1 + 5 * k;
      Record& o = out[st.records++];
      o.label = (int32_t)r[0];
      o.score = r[1];
      o.area = r[2];
      o.cx = r[3];
      o.cy = r[4];
      o.stream = stream;
      o.frame = fid;
      o.ts = ts;
    }
  }
  return st;
}

}  // namespace ssa
