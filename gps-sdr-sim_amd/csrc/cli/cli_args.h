/* cli_args.h — the reference command line (gpssim.c:1650-1852) parsed into gss_opts_t; the
   declarations (gss_cli_t, gss_cli_parse, gss_cli_usage) are part of the C ABI in gpssim_amd.h. */
#ifndef GSS_CLI_ARGS_H
#define GSS_CLI_ARGS_H
#include "gpssim_amd.h"
#endif
