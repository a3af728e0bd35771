// F = 16 instantiation of the templated kernels (one translation unit per F so the
// three variants compile in parallel).
#include "kernels_impl.h"
namespace msw {
MSW_INSTANTIATE(1)
}  // namespace msw
