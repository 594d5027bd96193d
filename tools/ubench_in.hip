#define SPX_FQ2_INLINE_MUL 1
#define SFX in
#include "ubench_kern.hpp"
