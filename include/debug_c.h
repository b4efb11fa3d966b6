/* debug_c.h -- ICB/debug_c.h: debug_c, declared in arpack_hip.h */
#ifndef ARPACK_HIP_ICB_DEBUG_C_H
#define ARPACK_HIP_ICB_DEBUG_C_H
#include "arpack_hip.h"
#endif
