// F = 64 instantiation of the templated kernels (one translation unit per F so the
// three variants compile in parallel).
#include "kernels_impl.h"
namespace msw {
MSW_INSTANTIATE(4)
}  // namespace msw
