/* debug_c.hpp -- ICB/debug_c.hpp: the C++ spelling of debug_c (arpack_hip.h) */
#ifndef ARPACK_HIP_ICB_DEBUG_C_HPP
#define ARPACK_HIP_ICB_DEBUG_C_HPP
#include "arpack_hip.h"
#endif
