/*
 * stat_c.hpp -- ICB/stat_c.hpp: C++ callers read the counters through
 * references (ICB/stat_c.hpp:9-18); this overload forwards to the C entry point
 * stat_c(a_int*, ..., float*) of arpack_hip.h.
 */
#ifndef ARPACK_HIP_ICB_STAT_C_HPP
#define ARPACK_HIP_ICB_STAT_C_HPP
#include "arpack_hip.h"

inline void stat_c(a_int& nopx, a_int& nbx, a_int& nrorth, a_int& nitref, a_int& nrstrt,
                   float& tsaupd, float& tsaup2, float& tsaitr, float& tseigt, float& tsgets,
                   float& tsapps, float& tsconv, float& tnaupd, float& tnaup2, float& tnaitr,
                   float& tneigh, float& tngets, float& tnapps, float& tnconv, float& tcaupd,
                   float& tcaup2, float& tcaitr, float& tceigh, float& tcgets, float& tcapps,
                   float& tcconv, float& tmvopx, float& tmvbx, float& tgetv0, float& titref,
                   float& trvec) {
    stat_c(&nopx, &nbx, &nrorth, &nitref, &nrstrt, &tsaupd, &tsaup2, &tsaitr, &tseigt, &tsgets,
           &tsapps, &tsconv, &tnaupd, &tnaup2, &tnaitr, &tneigh, &tngets, &tnapps, &tnconv,
           &tcaupd, &tcaup2, &tcaitr, &tceigh, &tcgets, &tcapps, &tcconv, &tmvopx, &tmvbx,
           &tgetv0, &titref, &trvec);
}
#endif
