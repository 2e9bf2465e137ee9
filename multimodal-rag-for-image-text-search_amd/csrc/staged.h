// staged.h — the device halves of K13 / K14 over bytes a caller has already staged: csrc/files.hip's
// host threads write the unstuffed entropy-coded segments and the inflated scanlines of a group
// into one pinned arena while the GPU works on the previous group, so the decode call does no
// per-file host work (no second parse, no unstuff, no copy into a staging buffer): descriptors,
// one copy per kind and the launches. Internal to the library (the C ABI is include/mrag.h).
#pragma once

#include <cstdint>

#include "jpeg_parse.h"

namespace mrag_stage {

// Stage bytes of one entropy-coded segment of len raw bytes, as K13 lays a batch out: the
// unstuffed bytes (<= len) at a 16-byte boundary, zero to the next one, then 16 bytes of slack.
inline int64_t jpeg_seg_stage_bytes(int64_t len) { return (len + 15) / 16 * 16 + 16; }

// n parsed JPEGs whose segments, in file then segment order, sit in stage[0 .. bytes) at the
// offsets jpeg_seg_stage_bytes gives, nbits[q] = 8 x the unstuffed length of segment q.
struct JpegStaged {
  const mrag_jpeg::Parsed* const* P;
  const uint8_t* stage;
  int64_t bytes;
  const uint32_t* nbits;
};
int jpeg_decode_staged(const JpegStaged& st, int32_t n, uint8_t* out, const int64_t* out_offsets, int32_t device,
                       void* stream);

// n PNGs' filtered scanlines at stage + raw_off[i] (inside stage[0 .. bytes)); dims as
// mrag_png_unfilter's (w, h, bytes per pixel per image).
int png_unfilter_staged(const uint8_t* stage, int64_t bytes, const int64_t* raw_off, const int32_t* dims, int32_t n,
                        uint8_t* out, const int64_t* out_offsets, int32_t device, void* stream);

}  // namespace mrag_stage
