#define SFX nl
#include "ubench_kern.hpp"
