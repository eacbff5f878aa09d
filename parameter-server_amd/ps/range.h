// ps/range.h — a half-open key range [begin, end) (reference src/ps/Range.h).
#pragma once
#include <cstdint>

namespace ps {

struct Range {
  Range() : Range(0, 0) {}
  Range(uint64_t b, uint64_t e) : begin(b), end(e) {}
  uint64_t size() const { return end - begin; }
  uint64_t begin;
  uint64_t end;
};

}  // namespace ps
