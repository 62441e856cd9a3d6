/* cli_args.h — the reference command line (gpssim.c:1650-1852) parsed into gss_opts_t. */
#ifndef GSS_CLI_ARGS_H
#define GSS_CLI_ARGS_H
#include "gpssim_amd.h"
typedef struct {
    gss_opts_t opt;
    char nav_file[256], motion_file[256], out_file[256];
} gss_cli_t;
/* Returns 0 to run, 1 after printing usage/errors (caller exits with status 1). */
int gss_cli_parse(int argc, char **argv, gss_cli_t *cli);
void gss_cli_usage(void);
#endif
