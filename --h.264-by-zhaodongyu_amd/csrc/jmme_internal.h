// jmme_internal.h -- kernel parameter block and launch helpers (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "jmme.h"

namespace jmme {

constexpr int kMaxLists = 2;
constexpr int kMaxRefs = 32;
constexpr int kKey32MaxRange = 44;   // (2R+1)^2 < 2^13 spiral ranks fit the 32-bit key
constexpr int kWG = 256;             // 4 waves of 64

struct KParams {
  const uint8_t *cur;                 // 8-bit current picture
  const uint8_t *const *refs;         // device table [kMaxLists*kMaxRefs] of 8-bit reference planes
  int pitch;                          // bytes per row (cur and refs)
  int width, height;                  // picture size (pels); reads clamp into it
  const jmme_mb_req *req;             // n units
  jmme_block_res *out;                // n * JMME_NSLOT
  int n;
  int mode;                           // JMME_FULL_SEARCH / JMME_FAST_FULL_SEARCH
  int max_mvd;                        // p_Vid->max_mvd (FFS gate)
  int lds_range;                      // largest search range in the launch (LDS sizing)
  unsigned *defer_count;              // units whose 32-bit keys saturated
  int *defer_list;
  const int *unit_list;               // optional indirection (deferred pass)
  const unsigned *unit_count;         // device count for the indirection
  unsigned *status;                   // bit 0: unit with range > lds_range; bit 1: sub-pel FS centre
  uint32_t *debug_words;              // debug: unit 0's first staged window (rows x wp words)
  unsigned long long *stamps;         // diagnostic builds (JMME_STAMPS): per-unit phase clocks
};

size_t units_lds_bytes(int lds_range);
hipError_t launch_units(const KParams &p, bool key32, int grid, hipStream_t s);

}  // namespace jmme
