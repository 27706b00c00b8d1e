// kp_sort.hip -- the radix sort behind the per-key posting-list build (tail.h k_kp_* /
// geobpe.hip tail_build): the live pairs (key id, token slot) sorted by key, stable, so each
// key's pairs form one run in slot order.  hipCUB's onesweep radix sort (rocPRIM) in a
// translation unit of its own (its templates would triple the main unit's compile time).
//
// The alternative to the default build, which counts and places every live pair with a
// returning global atomic on its key's list counter (k_kp_fill: ~25 M atomics, 4.7 GB of
// memory-side traffic and 1.46 ms at the C3 middle-regime switch).  The sorted runs place
// every pair with plain loads and stores, but the sort over every residue slot plus its
// scratch cost more end to end (C3 default run 25.3k vs 28.6k merges/s), so it is the A/B
// leg (GEOBPE_KP_ATOMIC=0), not the default.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstddef>
#include <cstdint>

namespace gb {

// temp == nullptr: *temp_bytes = the scratch the sort needs.  Keys are sorted on bits
// [0, end_bit); keys past the live ones carry all-ones in those bits and sort last.
hipError_t kp_sort_pairs(void* temp, size_t* temp_bytes, const int32_t* keys_in, int32_t* keys_out,
                         const int32_t* vals_in, int32_t* vals_out, int64_t n, int end_bit, hipStream_t s) {
  return hipcub::DeviceRadixSort::SortPairs(temp, *temp_bytes, reinterpret_cast<const uint32_t*>(keys_in),
                                            reinterpret_cast<uint32_t*>(keys_out), vals_in, vals_out, (int)n, 0,
                                            end_bit, s);
}

}  // namespace gb
