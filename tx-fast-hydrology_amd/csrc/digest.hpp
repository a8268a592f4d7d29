// Row digest of fetched outputs (the drop-in API's edit detector): the sum mod 2^64 over j of
//     t = (bits(row[j]) ^ (j * kDigestK1)) * kDigestK2;  t ^ (t >> 29)
// The term is a bijection of the element's bits for a fixed j, so changing any one element
// always changes the digest; the sum is order-free, so the device (kernels.hip row_digests, one
// workgroup per row) and the host (digest.cc, threads over column blocks) form the same value.
#pragma once

#include <cstdint>

namespace mcr {

constexpr uint64_t kDigestK1 = 0x9E3779B97F4A7C15ull;
constexpr uint64_t kDigestK2 = 0xD6E8FEB86659FD93ull;

// host form of the term (the device form is kernels.hpp digest_term: same constants)
inline uint64_t digest_term(uint64_t bits, uint64_t j) {
    uint64_t t = (bits ^ (j * kDigestK1)) * kDigestK2;
    return t ^ (t >> 29);
}

// out[r] = digest of rows[r][0 .. n) for r < nrows (a small persistent thread pool)
void host_digest_rows(const double* const* rows, int64_t nrows, int64_t n, uint64_t* out);

}  // namespace mcr
