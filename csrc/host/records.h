// Native unpack of the device's packed per-frame records (host side of K10, SURVEY.md
// §2.5): the per-step collect of the serving pipeline (parallel/dp.py) at small batches is
// host-bound on numpy call overhead, not on data (batch 1: ~30 us of numpy per step for two
// records; the reference builds its records in Python per contour, sem_seg_server.py:164-195).
#pragma once
#include <cstdint>

namespace ssa {

// numpy RECORD_DTYPE (runtime/results.py): 40 bytes, naturally aligned fields
struct Record {
  int32_t label;
  float score, area, cx, cy;
  int32_t stream;
  int64_t frame;
  double ts;
};
static_assert(sizeof(Record) == 40, "RECORD_DTYPE layout");

struct UnpackStats {
  int64_t records = 0;     // rows written
  int64_t overflow = 0;    // frames whose count was negative (more than K contours passed)
  int64_t pool_lost = 0;   // frames whose count was NaN (root pool exhausted: no records)
};

// packed: F rows of (1 + 5K) floats [count | K x (label, score, area, cx, cy)]; meta: F rows
// of (frame id, stream, capture ts) doubles. Writes the frames' records in push order into
// out (capacity cap rows; F * K always suffices).
UnpackStats unpack_records(const float* packed, int64_t F, int K, int64_t row_stride,
                           const double* meta, Record* out, int64_t cap);

}  // namespace ssa
