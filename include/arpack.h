/*
 * arpack.h -- the reference's ICB header name (ICB/arpack.h:10-21), so a C
 * caller written against arpack-ng builds unchanged against libarpack_hip.so:
 * every *aupd_c / *eupd_c entry point is declared in arpack_hip.h.
 */
#ifndef ARPACK_HIP_ICB_ARPACK_H
#define ARPACK_HIP_ICB_ARPACK_H
#include "arpack_hip.h"
#endif
