// Host-side argument validation of the C-ABI (include/polarldpc.h) under
// AddressSanitizer + UBSan ("ASan on the C-ABI shim in CPU tests").
// Built by tests/asan/Makefile against an ASan build of libpolarldpc.so (host
// code instrumented with -Xarch_host -fsanitize=...; device code unchanged) and
// run on a machine without a GPU: every bad argument must come back as
// PL_EINVAL / PL_EUNSUPPORTED with a message, valid plans must fail cleanly on
// the missing device (no leak, no crash), and no path may touch memory it
// does not own.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/polarldpc.h"

static int failures = 0;
#define EXPECT(cond)                                                              \
    do {                                                                          \
        if (!(cond)) {                                                            \
            std::fprintf(stderr, "FAIL %s:%d: %s (%s)\n", __FILE__, __LINE__, #cond, \
                         pl_last_error());                                        \
            ++failures;                                                           \
        }                                                                         \
    } while (0)

int main() {
    pl_plan* p = reinterpret_cast<pl_plan*>(0x1);
    std::vector<uint8_t> mask(1024, 0);
    for (int j = 0; j < 512; ++j) mask[j] = 1;
    // polar plan arguments (reference asserts, src/polar/decoder.py:17-18, 194-196)
    EXPECT(pl_polar_plan_create(1024, 512, mask.data(), 8, 0, nullptr) == PL_EINVAL);
    EXPECT(pl_polar_plan_create(1000, 500, mask.data(), 8, 0, &p) == PL_EINVAL && p == nullptr);
    EXPECT(pl_polar_plan_create(1024, 0, mask.data(), 8, 0, &p) == PL_EINVAL);
    EXPECT(pl_polar_plan_create(1024, 2048, mask.data(), 8, 0, &p) == PL_EINVAL);
    EXPECT(pl_polar_plan_create(1024, 511, mask.data(), 8, 0, &p) == PL_EINVAL);  // mask has 512 info bits
    EXPECT(pl_polar_plan_create(1024, 512, nullptr, 8, 0, &p) == PL_EINVAL);
    EXPECT(pl_polar_plan_create(1024, 512, mask.data(), -1, 0, &p) == PL_EINVAL);
    EXPECT(pl_polar_plan_create(1024, 512, mask.data(), 65537, 0, &p) == PL_EUNSUPPORTED);  // lists above 65536
    EXPECT(pl_polar_plan_create(32768, 512, mask.data(), 65536, 0, &p) == PL_EUNSUPPORTED);  // L * N > 2^30 (checked before the mask)
    EXPECT(pl_polar_plan_create(1 << 16, 8, mask.data(), 8, 0, &p) == PL_EINVAL);
    EXPECT(std::strlen(pl_last_error()) > 0);
    // a valid plan on a machine without a device: a clean device error, no leak
    int rc = pl_polar_plan_create(1024, 512, mask.data(), 8, 0, &p);
    EXPECT(rc == PL_OK || rc == PL_EHIP || rc == PL_ENOMEM);
    if (rc == PL_OK) pl_plan_destroy(p);
    // LDPC plan arguments
    std::vector<int32_t> rp = {0, 3, 6}, ci = {0, 1, 2, 1, 2, 3};
    EXPECT(pl_ldpc_plan_create(2, 4, rp.data(), ci.data(), 7, 20, 1, 1.0, 0, &p) == PL_EINVAL);
    EXPECT(pl_ldpc_plan_create(2, 4, rp.data(), ci.data(), PL_LDPC_BP, 0, 1, 1.0, 0, &p) == PL_EINVAL);
    EXPECT(pl_ldpc_plan_create(2, 4, nullptr, ci.data(), PL_LDPC_BP, 20, 1, 1.0, 0, &p) == PL_EINVAL);
    std::vector<int32_t> bad_ci = {0, 1, 4, 1, 2, 3};  // column out of range
    EXPECT(pl_ldpc_plan_create(2, 4, rp.data(), bad_ci.data(), PL_LDPC_BP, 20, 1, 1.0, 0, &p) == PL_EINVAL);
    std::vector<int32_t> desc_ci = {0, 2, 1, 1, 2, 3};  // not ascending within a check
    EXPECT(pl_ldpc_plan_create(2, 4, rp.data(), desc_ci.data(), PL_LDPC_BP, 20, 1, 1.0, 0, &p) == PL_EINVAL);
    std::vector<int32_t> rp_bad0 = {1, 3, 6};
    EXPECT(pl_ldpc_plan_create(2, 4, rp_bad0.data(), ci.data(), PL_LDPC_BP, 20, 1, 1.0, 0, &p) == PL_EINVAL);
    std::vector<int32_t> rp_deg1 = {0, 1, 6}, ci_deg1 = {0, 0, 1, 2, 3, 3};
    ci_deg1 = {0, 0, 1, 2, 3};
    rp_deg1 = {0, 1, 5};
    EXPECT(pl_ldpc_plan_create(2, 4, rp_deg1.data(), ci_deg1.data(), PL_LDPC_MS, 20, 1, 1.0, 0, &p) ==
           PL_EUNSUPPORTED);  // reference MSDecoder: ValueError on a degree-1 check
    rc = pl_ldpc_plan_create(2, 4, rp.data(), ci.data(), PL_LDPC_BP, 20, 1, 1.0, 0, &p);
    EXPECT(rc == PL_OK || rc == PL_EHIP || rc == PL_ENOMEM);
    if (rc == PL_OK) pl_plan_destroy(p);
    // decode / workspace arguments
    double llr[8] = {0};
    uint8_t bits[8] = {0};
    int64_t ws = 0;
    EXPECT(pl_decode(nullptr, llr, 1, 8, bits, nullptr, nullptr) == PL_EINVAL);
    EXPECT(pl_decode_ws(nullptr, llr, 1, 8, bits, nullptr, nullptr, 0, nullptr) == PL_EINVAL);
    EXPECT(pl_plan_workspace_bytes(nullptr, 1, &ws) == PL_EINVAL);
    EXPECT(pl_plan_reserve(nullptr, 1, nullptr) == PL_EINVAL);
    EXPECT(pl_plan_release(nullptr, nullptr) == PL_EINVAL);
    int64_t ns = 0, nb = 0;
    EXPECT(pl_plan_workspace_stats(nullptr, &ns, &nb) == PL_EINVAL);
    EXPECT(pl_debug_set_plan_device(nullptr, 0) == PL_EINVAL);
    EXPECT(pl_plan_get_info(nullptr, nullptr) == PL_EINVAL);
    EXPECT(pl_plan_destroy(nullptr) == PL_OK);
    EXPECT(pl_polar_plan_set_crc(nullptr, 8, 0x1D) == PL_EINVAL);
    // frame-source / counter arguments
    EXPECT(pl_random_bits(1, 0, -1, 8, bits, nullptr) == PL_EINVAL);
    EXPECT(pl_random_bits(1, 0, 1, 8, nullptr, nullptr) == PL_EINVAL);
    EXPECT(pl_awgn_llr(nullptr, 0, 1, 1.0, 1, 0, llr, 8, nullptr) == PL_EINVAL);
    EXPECT(pl_awgn_llr(nullptr, 8, 1, 1.0, 1, 0, llr, 4, nullptr) == PL_EINVAL);
    EXPECT(pl_rayleigh_llr(nullptr, 8, 1, 1.0, 1, 0, nullptr, 8, nullptr) == PL_EINVAL);
    EXPECT(pl_bsc(nullptr, 8, 1, 1.5, 1, 0, bits, 8, nullptr) == PL_EINVAL);
    EXPECT(pl_crc_append(bits, 8, 1, 4, 8, 0x1D, nullptr) == PL_EINVAL);  // ld < k_data + crc_len
    EXPECT(pl_crc_append(bits, 40, 1, 4, 33, 0x1D, nullptr) == PL_EINVAL);
    EXPECT(pl_gf2_encode(nullptr, 4, 8, bits, 4, 1, bits, 8, nullptr) == PL_EINVAL);
    EXPECT(pl_count_errors(bits, 8, bits, 8, 8, 1, nullptr, nullptr) == PL_EINVAL);
    EXPECT(pl_polar_encode(nullptr, bits, 1, bits, nullptr) == PL_EINVAL);
    if (failures) {
        std::fprintf(stderr, "%d failure(s)\n", failures);
        return 1;
    }
    std::printf("capi argument validation: all checks passed\n");
    return 0;
}
