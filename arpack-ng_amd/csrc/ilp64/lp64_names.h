// ILP64 build (libarpack_hip64.so): the LP64 reference ABI entry points of every
// translation unit are renamed ahip_lp64_*; csrc/ilp64/ilp64.cpp then defines the
// reference names with a_int = int64_t (arpackdef.h.in:6-14 with INTERFACE64=1)
// as narrowing shims over them.  Force-included (-include) by the Makefile.
#pragma once
#define dsaupd_c ahip_lp64_dsaupd_c
#define dseupd_c ahip_lp64_dseupd_c
#define dsaupd_ ahip_lp64_dsaupd_
#define dseupd_ ahip_lp64_dseupd_
#define dnaupd_c ahip_lp64_dnaupd_c
#define dneupd_c ahip_lp64_dneupd_c
#define dnaupd_ ahip_lp64_dnaupd_
#define dneupd_ ahip_lp64_dneupd_
#define znaupd_c ahip_lp64_znaupd_c
#define zneupd_c ahip_lp64_zneupd_c
#define znaupd_ ahip_lp64_znaupd_
#define zneupd_ ahip_lp64_zneupd_
#define ssaupd_c ahip_lp64_ssaupd_c
#define sseupd_c ahip_lp64_sseupd_c
#define ssaupd_ ahip_lp64_ssaupd_
#define sseupd_ ahip_lp64_sseupd_
#define snaupd_c ahip_lp64_snaupd_c
#define sneupd_c ahip_lp64_sneupd_c
#define snaupd_ ahip_lp64_snaupd_
#define sneupd_ ahip_lp64_sneupd_
#define cnaupd_c ahip_lp64_cnaupd_c
#define cneupd_c ahip_lp64_cneupd_c
#define cnaupd_ ahip_lp64_cnaupd_
#define cneupd_ ahip_lp64_cneupd_
#define stat_c ahip_lp64_stat_c
#define debug_c ahip_lp64_debug_c
