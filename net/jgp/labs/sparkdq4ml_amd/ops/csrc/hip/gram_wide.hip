// K5-wide placeholder (filled in by the LDS-tiled SYRK).
#include "gram_wide.h"

#include <stdexcept>

namespace dq4ml {

int64_t gram_wide_workspace(int, int, int64_t) { return 0; }
void gram_wide(int, const void*, int64_t, int, int64_t, int, const float*, void*, int64_t, double*, hipStream_t) {
  throw std::runtime_error("gram_wide: not implemented yet");
}

}  // namespace dq4ml
