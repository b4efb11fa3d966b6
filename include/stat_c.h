/* stat_c.h -- ICB/stat_c.h: sstats_c / sstatn_c / cstatn_c / stat_c, declared in arpack_hip.h */
#ifndef ARPACK_HIP_ICB_STAT_C_H
#define ARPACK_HIP_ICB_STAT_C_H
#include "arpack_hip.h"
#endif
