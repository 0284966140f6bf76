// sg_match.hip — A4 signature matching (placeholder until the matcher lands).
#include "sg_internal.hpp"
using namespace sg;
struct sg_matcher { int dummy; };
extern "C" {
int sg_ac_compile(const uint8_t *, const uint32_t *, uint32_t, uint32_t, sg_matcher **) { set_error("not built yet"); return SG_E_UNSUPPORTED; }
int sg_dfa_compile(const uint8_t *, const uint32_t *, uint32_t, uint32_t, sg_matcher **) { set_error("not built yet"); return SG_E_UNSUPPORTED; }
int sg_matcher_info(const sg_matcher *, uint64_t *, uint32_t *, uint32_t *) { return SG_E_UNSUPPORTED; }
int sg_match(sg_matcher *, const uint8_t *, size_t, uint64_t *, uint32_t *, size_t, size_t *) { return SG_E_UNSUPPORTED; }
int sg_dev_match(sg_ctx *, sg_matcher *, const uint8_t *, size_t, sg_dev_hits *) { return SG_E_UNSUPPORTED; }
void sg_free(void *) {}
}
