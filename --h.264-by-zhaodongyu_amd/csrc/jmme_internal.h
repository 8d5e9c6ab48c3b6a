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
constexpr int kStampWGs = 4096;      // diagnostic builds: per-workgroup records
constexpr int kCountWords = 16;      // KParams::counts; two sets, each launch's plan kernel zeroes the other

// One work item of the search kernels: the partitions of one MB x ref unit
// that share a search window AND a predictor/lambda (one SAD sweep serves all
// of them).  Built on the device by the plan kernel from the unit requests.
struct Item {
  unsigned long long gmask;   // partitions (slots) served; 0 = refused item (status set)
  int rs;                     // FFS: the members' own search range (<= R; positions beyond ring rs
                              // are not theirs, except a pre-seeded (0,0))
  int pad0;
  int u;                      // unit index
  int16_t mb_x, mb_y;
  int16_t cqx, cqy;           // window centre (qpel, on the integer grid)
  int16_t R, flags;           // window range; flags: kItemChk00 | kItemPreseed
  int16_t px, py;             // predictor (qpel)
  int lam;                    // lambda_factor
  int ref;                    // list * kMaxRefs + ref_idx
  int pad;
};
static_assert(sizeof(Item) == 48, "Item layout");
constexpr int kItemChk00 = 1;     // slot 0 takes check_for_00 (me_fullsearch.c:61)
constexpr int kItemPreseed = 2;   // FFS pos00 pre-seed (me_fullfast.c:640-648)
constexpr int kItemSlow64 = 4;    // lambda beyond the 32-bit keys: exact per-partition search

// 32-bit keys are cost << 11 | rank >> 2 (21-bit cost field).  Every partition
// but 16x16 stays exact while 32*32640 + lambda*74 < 2^21; the 16x16 key
// saturates instead (and an all-saturated 16x16 is searched again exactly).
constexpr uint32_t kMaxLambda32 = 14225;

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
  int key32;                          // plan: route items to the 32-bit list (else all to the 64-bit list)
  Item *items;                        // [item_cap]: unit u's first group at u, further groups from n on
  unsigned item_cap;
  unsigned *counts;                   // kCountWords: [0] further groups, [1] unused, [2] status,
                                      // [8 + x] XCD x's item tickets (item kernel)
  unsigned *counts_next;              // the other set: zeroed by the plan kernel for the next launch
                                      // (no memset launch per search)
  uint32_t *debug_words;              // debug: unit 0's first staged window (rows x wp words)
  unsigned long long *stamps;         // diagnostic builds (JMME_STAMPS): per-unit phase clocks
  int hbd;                            // 16-bit planes (pitch in samples): the 64-bit-key v_sad_u16 instance
  int chunk;                          // item kernel: consecutive items dealt to one XCD (>= 1)
  int rot;                            // ... the XCD of chunk (8 r + s) is (s - r / rot) mod 8 (0: s)
};
// status bits (counts[2]): bit 0 range > lds_range, bit 1 sub-pel centre, bit 2 refine lost a winner

// Low-latency form for small batches (a speculative batch after a failed
// guess is one or two macroblocks): items built on the host, each item's
// window split into 16x16-position tiles, one workgroup per (item, tile)
// storing its exact per-partition keys; a second launch takes the minimum over
// tiles and writes the results (mapped host memory).
struct SmallItem {
  const uint8_t *ref;         // the item's 8-bit reference plane
  unsigned long long gmask;   // partitions (slots) served
  int u;                      // unit index (result row)
  int16_t mb_x, mb_y;
  int16_t cqx, cqy;           // window centre (qpel, integer grid)
  int16_t R, rs;              // window range; FFS: the members' own range (<= R)
  int16_t px, py;             // predictor (qpel)
  int16_t flags;              // kItemChk00 | kItemPreseed
  uint16_t bmask;             // 4x4 blocks the served partitions cover (bit by*4+bx)
  int lam;
  int pad2;
};
static_assert(sizeof(SmallItem) == 48, "SmallItem layout");

constexpr int kSmallInline = 32;   // items a small launch carries in its kernel arguments

struct SmallParams {
  const uint8_t *cur;
  int pitch, width, height;           // pitch in pels (16-bit pels when hbd)
  int mode, max_mvd;
  int hbd;                            // SourceBitDepthLuma > 8: 16-bit planes (v_sad_u16)
  const SmallItem *items;             // n_items (device-readable: host-mapped pinned memory)
  int n_items;
  int tiles;                          // tiles per item side: ceil((2 * max R + 1) / 16)
  unsigned long long *keys;           // [n_items][tiles^2][JMME_NSLOT] per-tile keys
  int4 *info;                         // [n_items] gmask lo/hi, centre, unit, for the finish launch (device memory)
  jmme_block_res *out;                // [units * JMME_NSLOT] (host-mapped); only searched slots written
  // latency form: the first n_inline items travel in the kernel arguments (no
  // read of host memory before the first load), the per-tile keys go straight
  // to host-mapped memory and the host takes the minimum over tiles (no finish launch)
  int host_finish;
  int n_inline;
  SmallItem inl[kSmallInline];
};
constexpr int kSmallTile = 16;
hipError_t launch_search_small(const SmallParams &p, hipStream_t s);
// chained partition searches (jmme_search_mbs_chains): one workgroup per chain
constexpr int kChainInline = 8;     // chains per launch (kernel arguments)
constexpr int kChainMaxR = 44;      // largest window range the staged LDS window holds
struct ChainParams {
  const uint8_t *cur;
  const uint8_t *const *refs;       // device reference table
  int pitch, width, height;
  int mode, max_mvd, n, max_r;      // max_r: largest window range of the launch (LDS sizing)
  int hbd;                          // 16-bit planes (SourceBitDepthLuma 9..14): v_sad_u16 instantiation
  jmme_chain_res *res;              // [n][JMME_CHAIN_MAX_STEPS] (host-mapped)
  // in-chain SubPelME (jmme_search_mbs_chains_sp); subs == nullptr: integer-pel chains
  const uint8_t *const *subs;       // device sub-image table [list * kMaxRefs + ref]
  int sub_pitch;
  size_t plane_stride;
  jmme_block_res *sp_res;           // [n][JMME_CHAIN_MAX_STEPS] (host-mapped)
  uint32_t *done;                   // [n] (host-mapped): chain i stores seq behind its last result (or nullptr)
  uint32_t seq;
  jmme_chain chains[kChainInline];
  jmme_subpel_req sp[kChainInline]; // per chain: the SubPelME parameters
};
size_t chain_lds_bytes(int max_r, bool hbd = false);
hipError_t launch_search_chains(const ChainParams &p, hipStream_t s);

size_t items_lds_bytes(int lds_range, bool hbd = false);
// plan (unit requests -> items), then the persistent 32-bit and 64-bit item
// kernels; ev0/ev1 (optional) bracket the main search kernel
hipError_t launch_search(const KParams &p, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1);

}  // namespace jmme
