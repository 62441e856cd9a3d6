/*
 * gpssim_amd.h — C ABI of the MI355X-native GPS L1 C/A baseband synthesiser.
 *
 * The reference (TheShinning/gps-sdr-sim) has no plugin/FFI API: its hot path is inline code in
 * main() (gpssim.c:2190-2288) operating on locals chan[MAX_CHAN], gain[], iq_buff, iq8_buff, delt,
 * iq_buff_size and data_format (gpssim.c:1686-1716).  The seam this library exports is therefore
 * "synthesise K consecutive 0.1 s blocks given per-block channel parameters" (SURVEY.md §8b), plus
 * the host control plane that produces those parameters (gpssim.c:1672-2353 minus the sample loop).
 *
 * Two layers, one shared library (libgpssim_amd.so):
 *   1. Device layer (gss_dev_*, gss_synth_*): the hot path.  Replaces the per-sample loop
 *      gpssim.c:2190-2264 and the quantise/pack epilogue gpssim.c:2257-2288.  Plain pointers and
 *      sizes only; results are stream-ordered on the caller's HIP stream.
 *   2. Host layer (gss_scn_*): ephemeris parsing, 10 Hz range/Doppler refresh, nav message and
 *      channel allocation, and the exact carrier-phase planner.  Replaces gpssim.c:1672-2188 and
 *      2290-2353 (everything in main() around the sample loop).
 *
 * Error convention: every entry point returns 0 on success and a negative GSS_E* code on failure;
 * gss_last_error() returns a human-readable message for the calling thread.  Nothing here calls
 * exit(); the CLI (gps-sdr-sim) turns a failure into the reference's fprintf(stderr,…); exit(1).
 * Threading: a gss_dev / gss_scn handle is not thread-safe; use one host thread per GPU.
 */
#ifndef GPSSIM_AMD_H
#define GPSSIM_AMD_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GSS_MAXCH      16    /* MAX_CHAN, gpssim.h:16 */
#define GSS_CA_LEN     1023  /* CA_SEQ_LEN, gpssim.h:36 */
#define GSS_CA_WORDS   32    /* 1023 chips packed 32 per uint32 (bit j%32 of word j/32) */
#define GSS_NAV_WORDS  60    /* N_DWRD, gpssim.h:33 */

/* data formats: -b 1 / 8 / 16 (SC01/SC08/SC16, gpssim.h:77-79) */
#define GSS_FMT_SC01   1
#define GSS_FMT_SC08   8
#define GSS_FMT_SC16   16

#define GSS_OK           0
#define GSS_E_ARG       -1   /* invalid argument */
#define GSS_E_HIP       -2   /* HIP runtime error */
#define GSS_E_NOMEM     -3   /* allocation failed */
#define GSS_E_IO        -4   /* file open/read/write failed */
#define GSS_E_INPUT     -5   /* invalid input data (RINEX, motion file, start time …) */
#define GSS_E_STATE     -6   /* call out of order / exhausted */
#define GSS_E_NODEV     -7   /* no GPU / kernel image unavailable */
#define GSS_E_RANGE     -8   /* nav-word index ran past dwrd[59] (gpssim.c:2229-2232 overflow) */

/* ------------------------------------------------------------------------------------------ */
/* Per (block, channel) parameters: everything the sample loop reads.        */
/* ------------------------------------------------------------------------------------------ */
typedef struct gss_chan_blk {
    double  carr0;      /* chan[i].carr_phase at the block's first sample [cycles], FLOAT_CARR_PHASE
                           (gpssim.h:4).  Carried across blocks by the exact planner (gss_scn_*).   */
    double  carr_step;  /* chan[i].f_carr * delt, re-multiplied each sample in gpssim.c:2245       */
    double  code0;      /* chan[i].code_phase after computeCodePhase (gpssim.c:1334) [chips]       */
    double  code_step;  /* chan[i].f_code * delt (gpssim.c:2212)                                   */
    int32_t icode;      /* gpssim.c:1342 */
    int32_t ibit;       /* gpssim.c:1339 */
    int32_t iword;      /* gpssim.c:1336 */
    int32_t gain;       /* gain[i] (gpssim.c:2186), scaled by 2^7                                 */
    int32_t ca_tbl;     /* row of the ca_bits table (normally prn-1)                               */
    int32_t nav_tbl;    /* row of the dwrd table (chan[i].dwrd version)                            */
} gss_chan_blk_t;       /* 56 bytes; blocks are laid out [nblk][GSS_MAXCH], first nch[b] valid     */

/* ------------------------------------------------------------------------------------------ */
/* Device layer                                                                                */
/* ------------------------------------------------------------------------------------------ */
typedef struct gss_dev gss_dev;

/* Open device `ordinal` (hipSetDevice).  Fails with GSS_E_NODEV when no GPU is visible.       */
int gss_dev_open(gss_dev **out, int ordinal);
int gss_dev_close(gss_dev *d);

/* Pre-size both anchor sets for batches of up to `max_blocks` blocks of `n_per_blk` samples,
   so that the synthesis calls perform no allocation (graph-capturable).                       */
int gss_dev_reserve(gss_dev *d, int max_blocks, int n_per_blk);

/* Bytes of output one block produces: n*4 (SC16), n*2 (SC08), n/4 (SC01; n%4==0 required,
   see SURVEY.md Appendix A.4).  Returns 0 for an invalid format.                              */
size_t gss_block_bytes(int n_per_blk, int fmt);

/* Carrier checkpoints per block and channel: carr_ck[b][k][j] = exact carrier phase at sample
   (j * n_per_blk) / GSS_NCK of the block (j = 0 is carr0).  The host planner records them while
   it walks the carrier chain anyway (gss_scn_next); with them the GPU walks each block's carrier
   as GSS_NCK independent sub-chains.  Optional everywhere (NULL: the GPU walks whole blocks).   */
#define GSS_NCK 8

/* Synthesise nblk consecutive 0.1 s blocks.  ALL pointers are device pointers:
     blk      [nblk][GSS_MAXCH] channel parameters (first nch[b] of each row valid)
     nch      [nblk] active channel count per block (0..16)
     nch_max  host-side upper bound of nch[] over the batch (selects the kernel instance;
              blocks with fewer channels are padded with silent channels)
     carr_ck  optional [nblk][GSS_MAXCH][GSS_NCK] carrier checkpoints (see above)
     ca_bits  [n_ca][GSS_CA_WORDS] packed C/A chips (codegen, gpssim.c:132-171)
     nav      [n_nav][GSS_NAV_WORDS] 30-bit nav words (chan[i].dwrd, gpssim.c:1467-1547)
     out      nblk * gss_block_bytes(n_per_blk, fmt) bytes, exactly the bytes the reference
              fwrite()s for those blocks (gpssim.c:2276/2283/2287), concatenated in block order
     carr_end optional [nblk][GSS_MAXCH]: carrier phase after the block's last sample
     status   optional int32[1]: set non-zero if a nav-word index ran past 59
   stream is a hipStream_t (NULL = default stream).  Asynchronous; no host synchronisation.    */
int gss_synth_device(gss_dev *d, const gss_chan_blk_t *blk, const int32_t *nch, int nch_max,
                     const double *carr_ck, const uint32_t *ca_bits, int n_ca, const uint32_t *nav, int n_nav,
                     int nblk, int n_per_blk, int fmt, void *out, double *carr_end,
                     int32_t *status, void *stream);

/* gss_synth_device in its two stages, for pipelining consecutive batches (Stage A of batch k+1
   on one stream while Stage B renders batch k on another).  Stage A writes the exact state at
   every segment start of the batch into anchor set `set` (0 or 1, device-owned buffers); Stage
   B renders from that set.  Arguments as gss_synth_device; the caller orders the two on its
   streams (events) and passes Stage B the same blk/nch/nch_max/nblk/n_per_blk as Stage A of
   that set.  gss_synth_device == gss_anchor_device(set 0) then gss_render_device(set 0) on one
   stream.                                                                                     */
int gss_anchor_device(gss_dev *d, int set, const gss_chan_blk_t *blk, const int32_t *nch,
                      int nch_max, const double *carr_ck, int nblk, int n_per_blk,
                      double *carr_end, void *stream);
int gss_render_device(gss_dev *d, int set, const gss_chan_blk_t *blk, const int32_t *nch,
                      int nch_max, const uint32_t *ca_bits, int n_ca, const uint32_t *nav,
                      int n_nav, int nblk, int n_per_blk, int fmt, void *out, int32_t *status,
                      void *stream);

/* ---- certified linear fast path ------------------------------------------------------------
   For most blocks each channel's exact carrier and code trajectories stay so close to a 64-bit
   integer line that every sample's LUT cell, chip and code wrap can be read off the line.
   gss_linearize (host) finds the lines and proves that, block by block, with exact integer
   arithmetic; gss_synth_lin_device renders the proven blocks with integer steps only and sends
   the rest (fast[b] == 0) through the exact walking path (Stage A + Stage B).  Same bytes.     */
#define GSS_NGC 8                /* signed-gain schedule entries per block and channel        */
#define GSS_NPATCH 8             /* patched samples per block and channel                     */
typedef struct gss_lin {
    uint64_t x0, xs;             /* carrier line, 2^-64 cycle: x0 + p*xs mod 2^64              */
    uint64_t z0, zs;             /* code line, 2^-50 chip, unwrapped: floor((z0 + p*zs) / 2^50)
                                    = chips since the block's code wrap base; chip index is that
                                    mod 1023 and the k-th code wrap falls where it reaches 1023k */
    int64_t pdelta[GSS_NPATCH];  /* correction of sample ppos[i]'s packed I/Q term (exact minus
                                    what the kernel's render arithmetic reads there, both
                                    gain * codeCA * (cos + 2^22 sin), gpssim.c:2190-2256)      */
    int32_t gpos[GSS_NGC];       /* gain*dataBit (gpssim.c:2186, 2234) is gval[i] for samples   */
    int32_t gval[GSS_NGC];       /* gpos[i] <= p < gpos[i+1]; gpos[0] = 0, unused = INT32_MAX   */
    int32_t ppos[GSS_NPATCH];    /* patched samples, ascending (unused = INT32_MAX)             */
} gss_lin_t;                     /* 192 bytes, laid out [nblk][GSS_MAXCH]                      */

/* Lines and proofs for nblk blocks (host arrays; ca_bits = [n_ca][GSS_CA_WORDS] and nav =
   [n_nav][GSS_NAV_WORDS] rows as passed to the synth calls).  fast[b] = 1 if every channel of
   block b is certified (and the block's gains fit the packed accumulator), else 0.  Runs on
   `threads` host threads.                                                                     */
int gss_linearize(const gss_chan_blk_t *blk, const int32_t *nch, int nblk, int n_per_blk,
                  const uint32_t *ca_bits, int n_ca, const uint32_t *nav, int n_nav,
                  gss_lin_t *lin, int32_t *fast, int threads);

/* gss_linearize on the GPU: the same proofs and the same rows, byte for byte (the per-channel
   proof is csrc/common/gss_proof.h on both sides).  Device pointers; asynchronous on `stream`.
   gss_run proves with this call the slots of its planner-bound runs (rows ahead, slots of >= 1024
   blocks: the -b 1 runs) and on the host threads the others; GSS_RUN_PROOF=gpu / host / split
   (every other slot on the GPU) forces a mode.  One workgroup per block; a small launch spreads
   the channels over waves (GSS_PROOF_STRIDE=1 / 16 / 32 / 64 forces the shape, for tests).    */
int gss_linearize_device(gss_dev *d, const gss_chan_blk_t *blk, const int32_t *nch, int nblk,
                         int n_per_blk, const uint32_t *ca_bits, int n_ca, const uint32_t *nav,
                         int n_nav, gss_lin_t *lin, int32_t *fast, void *stream);

/* gss_synth_device over the certified fast path.  Device pointers as gss_synth_device, plus
   lin [nblk][GSS_MAXCH] and fast [nblk] from gss_linearize, and the exact path's block list
   fb_list [n_fb] (device; the indices b with fast[b] == 0, n_fb known on the host).  carr_ck
   (optional) feeds the exact path's Stage A.  No carr_end output.                             */
int gss_synth_lin_device(gss_dev *d, const gss_chan_blk_t *blk, const int32_t *nch, int nch_max,
                         const gss_lin_t *lin, const int32_t *fast, const int32_t *fb_list,
                         int n_fb, const double *carr_ck, const uint32_t *ca_bits, int n_ca,
                         const uint32_t *nav, int n_nav, int nblk, int n_per_blk, int fmt,
                         void *out, int32_t *status, void *stream);

/* min and max of (a + p*s) mod m over 0 <= p < n, exactly (the certificate's core; exported for
   tests).                                                                                      */
void gss_minmax_mod(uint64_t n, uint64_t m, uint64_t a, uint64_t s, uint64_t *mn, uint64_t *mx);
/* tests: the least p in [0, n) with (a + p s) mod m < w (n if none; UINT64_MAX for m = 0 or
   m >= 2^62, w = 0 or w > m) -- the proof's enumeration of ambiguous samples */
uint64_t gss_first_below(uint64_t n, uint64_t m, uint64_t a, uint64_t s, uint64_t w);
/* the proof's ambiguous samples: p in [1, n) with (a0 + p st) mod 2^lgB < w, ascending, up to
   cap in hit[]; their number, -1 if more, -2 on bad arguments (scan: one descent per hit, else
   the three-gap stepping the proofs use; both give the same list; exported for tests)        */
int gss_hits_mod(uint64_t n, uint64_t lgB, uint64_t a0, uint64_t st, uint64_t w, int64_t *hit,
                 int cap, int scan);

/* Same, from host buffers: uploads inputs, runs, downloads `out` (and carr_end if non-NULL),
   synchronises.  Convenience for the CLI and tests; the bench uses gss_synth_device().
   Without carr_end it linearises and takes the fast path (env GSS_PATH=walk: exact path
   only).                                                                                      */
int gss_synth_host(gss_dev *d, const gss_chan_blk_t *blk, const int32_t *nch,
                   const double *carr_ck, const uint32_t *ca_bits, int n_ca, const uint32_t *nav, int n_nav,
                   int nblk, int n_per_blk, int fmt, void *out, double *carr_end);

/* Kernel timing from HIP events recorded on the launch stream around every Stage A and Stage B
   launch (gss_synth_device, gss_anchor_device, gss_render_device; rings of the last 256 of
   each).  reset!=0 clears the rings (no sync); otherwise waits for the last launches and
   returns the number n of Stage B launches and the average duration [ms] of each stage.      */
int gss_dev_timing(gss_dev *d, int reset, int *n, float *ckpt_ms, float *synth_ms);
/* Same for the fast-path kernel of gss_synth_lin_device (its exact-path leftovers count as
   Stage A / Stage B launches above); the same reset clears it.                               */
int gss_dev_timing_lin(gss_dev *d, int *n, float *lin_ms);

/* ------------------------------------------------------------------------------------------ */
/* Host layer: scenario driver mirroring main() (gpssim.c:1672-2353)                           */
/* ------------------------------------------------------------------------------------------ */
typedef struct gss_opts {
    const char *nav_file;       /* -e  RINEX v2 navigation file (required)                     */
    const char *motion_file;    /* -u  user motion CSV / -g NMEA GGA (NULL: static)            */
    int    nmea;                /* 1 if motion_file is NMEA GGA (-g)                           */
    int    has_xyz;             /* -c given: xyz holds ECEF [m]                                */
    double xyz[3];
    int    has_llh;             /* -l given: llh holds lat [deg], lon [deg], height [m]        */
    double llh[3];
    double samp_freq;           /* -s [Hz], default 2.6e6                                      */
    int    data_format;         /* -b 1/8/16, default 16                                       */
    double duration;            /* -d [s]; <0 → default USER_MOTION_SIZE/10                    */
    int    has_start;           /* -t / -T given                                               */
    int    time_overwrite;      /* -T                                                          */
    int    start[6];            /* y m d hh mm ss (already validated & floor()ed by caller)     */
    double start_sec;
    int    iono_disable;        /* -i                                                          */
    int    verbose;             /* -v                                                          */
    int    user_motion_size;    /* USER_MOTION_SIZE (gpssim.h:19-21), 0 → 3000                 */
    int    quiet;               /* suppress the reference's stderr chatter (library use)       */
    int    carrier_int;         /* 1: the reference built without FLOAT_CARR_PHASE (gpssim.h:4):
                                   32-bit integer carrier in 2^-25 cycle, step
                                   (int)round(2^25 f_carr delt) (gpssim.c:1623-1626, 2175-2177,
                                   2201-2202, 2252).  CLI: --carrier=int (default float).  The
                                   rows then carry that integer chain as exact doubles, carr0 =
                                   (carr_phase mod 2^25) / 2^25 and carr_step = step / 2^25, whose
                                   IEEE recurrence is the integer one, so every kernel renders it
                                   unchanged.                                                   */
} gss_opts_t;

/* The reference command line (getopt "e:u:g:c:l:o:s:b:T:t:d:iv", gpssim.c:1650-1852) parsed
   into options, with the reference's validation messages on stderr.  Returns 0 to run, 1 after
   printing usage or an error (the reference then exits with status 1).  The strings opt points
   at live in the struct.                                                                       */
typedef struct gss_cli {
    gss_opts_t opt;
    char nav_file[256], motion_file[256], out_file[256];
} gss_cli_t;
int gss_cli_parse(int argc, char **argv, gss_cli_t *cli);
void gss_cli_usage(void);

typedef struct gss_scn_info {
    int    n_per_blk;           /* iq_buff_size = floor(fs/10) (gpssim.c:1877-1878)            */
    int    n_blocks;            /* numd-1: blocks the run writes (gpssim.c:2154)               */
    int    data_format;
    double samp_freq;           /* after rounding to a multiple of 10 Hz                       */
    double delt;                /* 1/samp_freq (gpssim.c:1881)                                 */
    int    week;  double sec;   /* g0 (start time)                                             */
    int64_t next_block;         /* run index of the next block gss_scn_next* produces          */
    int64_t rows_out;           /* blocks whose rows this handle produced (gss_scn_seek skips
                                   blocks without producing them)                              */
    int    carrier_int;         /* gss_opts_t.carrier_int                                      */
} gss_scn_info_t;

typedef struct gss_scn gss_scn;

/* Parse inputs, select ephemeris set and start time, allocate the first channels.
   On error returns GSS_E_* and *out stays NULL (message via gss_last_error()).               */
int gss_scn_open(gss_scn **out, const gss_opts_t *opt);
int gss_scn_info(const gss_scn *s, gss_scn_info_t *info);

/* Produce parameters for the next up to `max_blocks` blocks (in run order), including the
   exact carrier phase at each block start (planner runs on `threads` host threads).
   blk is [max_blocks][GSS_MAXCH], nch is [max_blocks], carr_ck (optional, may be NULL) is
   [max_blocks][GSS_MAXCH][GSS_NCK] carrier checkpoints.  *n_out = blocks produced (0 at end). */
int gss_scn_next(gss_scn *s, int max_blocks, gss_chan_blk_t *blk, int32_t *nch, double *carr_ck,
                 int *n_out, int threads);

/* ---- planning a time window without its prefix (multi-GPU: plan once, scatter) ----------------
   The carrier phase is the only state the sample loop carries across blocks (gpssim.c:2245-2250;
   the code state is recomputed every block, gpssim.c:1331-1345), and it is one chain per channel
   slot, restarted where allocateChannel re-initialises the slot (gpssim.c:1615-1626).  So a rank
   can produce its window's rows by itself (gss_scn_seek + gss_scn_next_deferred) and receive only
   the 16 slot carriers at its first block from the rank before it, which runs the chain over its
   own window (gss_carr_chain) and hands the end state on.                                     */
typedef struct gss_chain {       /* per (block, channel row): the carrier chain it continues     */
    int8_t  slot;                /* chan[] slot 0..15; -1 for padding rows                        */
    uint8_t reset;               /* 1: the slot's chain restarts at this block with `init`        */
    uint8_t pad[6];
    double  init;                /* carr_phase set by allocateChannel (valid when reset)          */
} gss_chain_t;                   /* 16 bytes, laid out [nblk][GSS_MAXCH] like the rows             */

/* gss_scn_next without the carrier chain: blk[].carr0 is left 0 and chain[] says which slot's
   chain each row continues; gss_carr_chain fills carr0 (and checkpoints) afterwards.  The
   handle's slot carriers (gss_scn_carrier) stay those at the first produced block, and
   gss_scn_next fails with GSS_E_STATE until gss_scn_set_carrier supplies the chain's end.       */
int gss_scn_next_deferred(gss_scn *s, int max_blocks, gss_chan_blk_t *blk, int32_t *nch,
                          gss_chain_t *chain, int *n_out, int threads);
/* The carrier chain over nblk consecutive blocks of deferred rows: carr[GSS_MAXCH] holds each
   slot's carrier phase at the first block's start on entry and after the last block on return;
   fills blk[].carr0 and, if carr_ck != NULL, the [nblk][GSS_MAXCH][GSS_NCK] checkpoints.
   carrier_int: the integer-carrier chain of gss_opts_t.carrier_int.  One slot per thread.    */
int gss_carr_chain(double *carr, gss_chan_blk_t *blk, const int32_t *nch,
                   const gss_chain_t *chain, int nblk, int n_per_blk, int carrier_int,
                   double *carr_ck, int threads);
/* The same chain with the blocks' walks run ahead of it, in parallel (the chain's serial part is
   then one partial cycle per block; gss_phase.h, "speculative block walk").
     gss_carr_chain_guess  each row's guesses: its start from the line of its slot (exact at the
                           slot's first block and at a reset) and up to GSS_SPEC_K - 1 segment
                           starts at wraps the line predicts, in[nblk][GSS_MAXCH] (padding: s 0)
     gss_carr_chain_starts the starts only, live rows left with k = 0: the walkers guess their
                           segment starts themselves and write them back into in[] (gss_run)
     gss_spec_host/device  the speculative walk of every row's segments: spec[nrow]; host
                           threads, or the GPU (device-visible pointers, async on stream; gss_run;
                           one lane per segment, rows channel-major for a multiple of GSS_MAXCH)
     gss_carr_chain_spec   the chain: as gss_carr_chain without checkpoints, each block's end from
                           its true start and its speculative walk (exact whether or not the
                           translation applies); *n_hit counts the blocks where it did.        */
#ifndef GSS_SPEC_T_DEFINED
#define GSS_SPEC_T_DEFINED
#ifndef GSS_SPEC_K
#define GSS_SPEC_K 32                   /* segments per block (8 before round 6: the GPU walks
                                          then took 1.19 ms per headline window, 0.88 with 16;
                                          with the row-shared cycle cache 0.65 with 16, 0.55
                                          with 32, 0.61 with 64: profiles/round6/spec_k/s6z) */
#endif
typedef struct gss_spec_in {           /* a row's guesses (host, gss_carr_chain_guess)          */
    double g, s;                       /* start guess, carr_step (0: padding row)               */
    int32_t k, pad;                    /* segments (1..GSS_SPEC_K; 0: not guessed yet)          */
    int64_t P[GSS_SPEC_K];             /* segment j >= 1 starts at sample P[j], a predicted wrap */
    double W[GSS_SPEC_K];              /* ... with post-wrap value W[j]                         */
} gss_spec_in_t;                       /* 24 + 16 GSS_SPEC_K bytes (536) */
typedef struct gss_spec_seg {
    double end, dlo, dhi;              /* end value, admissible translations of the start       */
    int64_t wrap_end;                  /* 1: the segment's last step wrapped                    */
} gss_spec_seg_t;
typedef struct gss_spec {              /* a row's speculative walk (GPU or host)                */
    int64_t p1;                        /* samples to the guess's first wrap (n: none)           */
    double w1;                         /* its post-wrap value                                   */
    gss_spec_seg_t seg[GSS_SPEC_K];
} gss_spec_t;                          /* 16 + 32 GSS_SPEC_K bytes (1040) */
#endif
int gss_carr_chain_guess(const double *carr, const gss_chan_blk_t *blk, const int32_t *nch,
                         const gss_chain_t *chain, int nblk, int n_per_blk, gss_spec_in_t *in);
int gss_carr_chain_starts(const double *carr, const gss_chan_blk_t *blk, const int32_t *nch,
                          const gss_chain_t *chain, int nblk, int n_per_blk, gss_spec_in_t *in);
/* The slots' carriers after the nblk blocks by the same lines: a prediction, the start of the
   next batch's guesses while this batch's chain is still pending (gss_run keeps two batches of
   walks in flight). */
int gss_carr_line_end(const double *carr, const gss_chan_blk_t *blk, const int32_t *nch,
                      const gss_chain_t *chain, int nblk, int n_per_blk, double *carr_end);
int gss_spec_host(gss_spec_in_t *in, int nrow, int n_per_blk, gss_spec_t *spec, int threads);
int gss_spec_device(gss_dev *d, gss_spec_in_t *in, int nrow, int n_per_blk, gss_spec_t *spec,
                    void *stream);
int gss_carr_chain_spec(double *carr, gss_chan_blk_t *blk, const int32_t *nch,
                        const gss_chain_t *chain, int nblk, int n_per_blk,
                        const gss_spec_in_t *in, const gss_spec_t *spec, int threads,
                        int *n_hit);
/* Records: each row's speculative walk folded into 72 bytes (gss_spec_rec_t: the interval of
   translations of its first post-wrap value that carry it through every segment, and of its
   predecessor's last translation that carry it from the predecessor's end), so that the chain
   needs neither the walks (1,040 B) nor the segment guesses (536 B) on the host (gss_run: the
   walks stay on the device and only the records cross the link).  The previous row of a row's
   slot chain in the batch is in[].pad (gss_carr_chain_starts / _guess set it; -1: none).
     gss_spec_records         the records from walks on the host
     gss_spec_records_device  walks and records on the GPU: in (host-visible rows, their
                              starts), d_in / d_spec (device scratch, nrow rows), rec
                              (host-visible); async on stream
     gss_carr_chain_records   the chain from the records (exact: a failed interval walks)   */
#ifndef GSS_SPEC_REC_DEFINED
#define GSS_SPEC_REC_DEFINED
typedef struct gss_spec_rec {
    double w1;                         /* post-wrap value at the guess's first wrap                */
    double slo, shi, sdd;              /* self: d0 = (true post-wrap value at p1) - w1 in [slo,
                                          shi] -> the row's last translation is d0 + sdd ...     */
    double end;                        /* ... and its end is end + (d0 + sdd)                      */
    double llo, lhi, ldd;              /* link: the previous row of the slot translated by d in
                                          [llo, lhi] -> this one's last translation is d + ldd    */
    int32_t p1;                        /* samples to the guess's first wrap                        */
    int32_t ok;                        /* bit 0: self record, bit 1: link record, bits 2..: the
                                          link's row distance (this row - in[].pad), which the
                                          chain checks against the slot's actual previous row  */
} gss_spec_rec_t;                      /* 72 bytes */
#endif
int gss_spec_records(const gss_spec_in_t *in, const gss_spec_t *spec, int nrow, int n_per_blk,
                     gss_spec_rec_t *rec, int threads);
int gss_spec_records_device(gss_dev *d, const gss_spec_in_t *in, int nrow, int n_per_blk,
                            gss_spec_in_t *d_in, gss_spec_t *d_spec, gss_spec_rec_t *rec,
                            void *stream);
int gss_carr_chain_records(double *carr, gss_chan_blk_t *blk, const int32_t *nch,
                           const gss_chain_t *chain, int nblk, int n_per_blk,
                           const gss_spec_rec_t *rec, int threads, int *n_hit);
/* Anchors: exact carrier values inside a block, by-products of the chain (the values at the
   segment starts its fix-up passed or walked), which the proofs start their exact carrier walks
   from (gss_linearize_ex / gss_linearize_device_ex) instead of from the block start.
     gss_carr_chain_anchored  gss_carr_chain_spec, also filling anch[nblk][GSS_MAXCH]
     gss_carr_anchors         the same anchors for rows whose carr0 any chain has set, in parallel
                              over blocks (the speculative walks of those rows, gss_spec_*)   */
typedef struct gss_carr_anchor {
    int32_t pos[GSS_SPEC_K];           /* sample positions within the block (-1: none); pos[0] 0 */
    double val[GSS_SPEC_K];            /* the reference's carr_phase at sample pos (val[0] carr0) */
} gss_carr_anchor_t;                   /* 12 GSS_SPEC_K bytes (384) */
int gss_carr_chain_anchored(double *carr, gss_chan_blk_t *blk, const int32_t *nch,
                            const gss_chain_t *chain, int nblk, int n_per_blk,
                            const gss_spec_in_t *in, const gss_spec_t *spec, int threads,
                            int *n_hit, gss_carr_anchor_t *anch);
int gss_carr_anchors(const gss_chan_blk_t *blk, const int32_t *nch, int nblk, int n_per_blk,
                     const gss_spec_in_t *in, const gss_spec_t *spec, gss_carr_anchor_t *anch,
                     int threads);
/* gss_linearize / gss_linearize_device with the anchors (anch [nblk][GSS_MAXCH], NULL: none;
   device memory for the _device form): the same rows, byte for byte, with shorter walks.      */
int gss_linearize_ex(const gss_chan_blk_t *blk, const int32_t *nch, int nblk, int n_per_blk,
                     const uint32_t *ca_bits, int n_ca, const uint32_t *nav, int n_nav,
                     const gss_carr_anchor_t *anch, gss_lin_t *lin, int32_t *fast, int threads);
int gss_linearize_device_ex(gss_dev *d, const gss_chan_blk_t *blk, const int32_t *nch, int nblk,
                            int n_per_blk, const uint32_t *ca_bits, int n_ca,
                            const uint32_t *nav, int n_nav, const gss_carr_anchor_t *anch,
                            gss_lin_t *lin, int32_t *fast, void *stream);
/* Links between a slot's consecutive rows, computed before the chain's start is known (the
   multi-rank planner runs them ahead of the baton; gpssim_amd/shard.py chain_speculated):
     gss_spec_links         for every row that continues its slot's chain in the batch, its
                            whole walk folded into one record from the previous row's
                            speculative end (its partial cycle to the first wrap walked from
                            there ahead of time, with the admissible translations)
     gss_carr_chain_linked  gss_carr_chain_spec's result, where a row whose predecessor's
                            translation held is one compare and two adds: the serial part is then
                            a few ns per row, plus the exact walks where a translation fails. */
typedef struct gss_spec_link {
    double lo, hi;                     /* the previous row translated by d in [lo, hi] (lo > hi:
                                          no record): this row translates too ...               */
    double dd, end;                    /* ... by d + dd, and ends at end + (d + dd)             */
} gss_spec_link_t;                     /* 32 bytes */
int gss_spec_links(const int32_t *nch, const gss_chain_t *chain, int nblk, int n_per_blk,
                   const gss_spec_in_t *in, const gss_spec_t *spec, gss_spec_link_t *link,
                   int threads);
int gss_carr_chain_linked(double *carr, gss_chan_blk_t *blk, const int32_t *nch,
                          const gss_chain_t *chain, int nblk, int n_per_blk,
                          const gss_spec_in_t *in, const gss_spec_t *spec,
                          const gss_spec_link_t *link, int threads, int *n_hit);
/* Move to run block `block` (>= the next block) without producing the blocks in between: only the
   30 s updates are replayed (nav frames, ephemeris steps, allocation), and the ranges of the
   block before the target (rho0 of computeCodePhase).  The slot carriers are unknown afterwards:
   gss_scn_next fails until gss_scn_set_carrier; gss_scn_next_deferred works.                */
int gss_scn_seek(gss_scn *s, int64_t block, int threads);
/* The planner's carrier per slot at the next block (get) / set it (after a seek).             */
int gss_scn_carrier(const gss_scn *s, double *carr);
int gss_scn_set_carrier(gss_scn *s, const double *carr);

/* Nav-word table rows produced so far ([n][GSS_NAV_WORDS]); valid until the next gss_scn_next. */
int gss_scn_nav_table(const gss_scn *s, const uint32_t **rows, int *n_rows);

/* Packed C/A codes for PRN 1..32 into out[32][GSS_CA_WORDS] (row prn-1).                      */
int gss_ca_table(uint32_t *out);

/* ---- the 30 s producers on the GPU ---------------------------------------------
   What the 30 s cadence produces for the sample loop -- the C/A chips (codegen, gpssim.c:132-171)
   and each channel's LNAV frame words with parity (generateNavMsg, gpssim.c:1467-1547) -- built
   on the device.  The host keeps what needs libm-exact doubles: ephemeris-to-subframe packing
   (eph2sbf, gpssim.c:490-665), allocation and ranges.  A nav-table row is described by its
   source: the frame's subframe data words, TOW count and week, and where its first ten words
   (the previous frame's subframe 5) come from.                                                */
#define GSS_NAV_HEAD_INIT   (-1)   /* rebuilt from sbf[4] with tow (a newly allocated channel) */
#define GSS_NAV_HEAD_GIVEN  (-2)   /* in head[] (the first row after a seek)                    */
typedef struct {
    uint32_t sbf[5][10];     /* subframe data words (no TOW/WN/parity) at the frame's update   */
    uint32_t tow;            /* g0.sec / 6: the TOW count before the first subframe            */
    uint32_t wn;             /* g0.week % 1024                                                  */
    int32_t  prev;           /* >= 0: row whose words 50..59 are this row's words 0..9, else
                                GSS_NAV_HEAD_INIT / GSS_NAV_HEAD_GIVEN                          */
    int32_t  next;           /* row continuing this one (its prev), or -1                       */
    uint32_t head[10];       /* words 0..9 for GSS_NAV_HEAD_GIVEN                               */
} gss_nav_src_t;             /* 256 bytes; row r of gss_scn_nav_table is built from source r   */

/* The sources of the rows of gss_scn_nav_table ([n], same order); next links within the table. */
int gss_scn_nav_sources(const gss_scn *s, const gss_nav_src_t **src, int *n_rows);
/* Rows [first, first + n) of a nav table from their sources src[0 .. n) (host: the producers'
   reference); rows before `first` must already be in rows (a source's prev may point there). */
int gss_nav_rows_host(const gss_nav_src_t *src, int first, int n, uint32_t *rows);
/* The same on the device (asynchronous on `stream`): src, rows are device pointers, src holds
   the sources of rows [first, first + n) at src[0 .. n); one lane per chain of rows.          */
int gss_nav_rows_device(gss_dev *d, const gss_nav_src_t *src, int first, int n, uint32_t *rows,
                        void *stream);
/* The packed C/A table of gss_ca_table built on the device into out[32][GSS_CA_WORDS].        */
int gss_ca_table_device(gss_dev *d, uint32_t *out, void *stream);

/* Wall time [s] the host planner spent so far (control plane + carrier chain).                */
double gss_scn_plan_seconds(const gss_scn *s);

int gss_scn_close(gss_scn *s);

/* ------------------------------------------------------------------------------------------ */
/* Streaming driver: the reference's block loop (gpssim.c:2154-2353) end to end               */
/* ------------------------------------------------------------------------------------------ */
/* Byte sink of gss_run: called in run order on the calling thread with the exact output bytes
   of `nblocks` consecutive blocks starting at run block `first_block` (what the reference
   fwrite()s for them).  Return 0 to continue, non-zero to stop the run (GSS_E_IO).            */
typedef int (*gss_sink_fn)(void *user, const void *bytes, size_t n, int64_t first_block,
                           int nblocks);

/* Run blocks [first_block, first_block + n_blocks) of scenario s (n_blocks < 0: to the end) on
   device d and stream their bytes to `sink`.  Planning (gss_scn_next on `threads` host
   threads, in its own thread), upload, both kernel stages, download into pinned buffers and the
   sink overlap; `batch` blocks per launch (capped at 256 MiB of output).  Blocks before
   first_block are planned (the carrier chain is serial) but not synthesised: a rank of a
   multi-GPU run passes its own range and writes at first_block * gss_block_bytes().           */
int gss_run(gss_dev *d, gss_scn *s, int64_t first_block, int64_t n_blocks, int batch,
            int threads, gss_sink_fn sink, void *user);

/* gss_run for one process of a multi-process run, planned once per node (no process plans another
   process's blocks): with carr_in set, the planner thread seeks to first_block (gss_scn_seek),
   produces the range's rows (gss_scn_next_deferred), calls carr_in for the 16 slot carriers at
   first_block (it may block until the process before has them), walks the carrier chain over
   the range (gss_carr_chain) and hands the end state to carr_out (if set) -- before the first
   batch renders.  Both callbacks return 0, or non-zero to abort the run (GSS_E_IO).
   opts == NULL or carr_in == NULL: gss_run (blocks before first_block planned and dropped).  */
typedef struct gss_run_opts {
    int (*carr_in)(void *user, double *carr);             /* [GSS_MAXCH], out                  */
    int (*carr_out)(void *user, const double *carr);      /* [GSS_MAXCH]                       */
    void *carr_user;
    /* Optional: the chain speculated across ranks.  Called twice (round 0: by the lines, round
       1: by an exact chain from the first prediction) before carr_in, with this range's map of
       the slot carriers, map[3 * GSS_MAXCH] = {start (the run's initial carriers when the range
       starts at block 0, else 0), add, reset}: the range takes x to reset ? add : (x + add) mod
       1 per slot.  It publishes the map to the ranks after this one and returns in start_out
       the composition of the maps of the ranks before it (gpssim_amd/shard.py compose_start).
       The walks then run before carr_in, and from carr_in to carr_out only the records' chain
       is left.  Exact whatever the predictions.  A rank that is given the
       callback but does not speculate (GSS_RUN_SPEC=0 or GSS_RUN_REC=0 in its environment, or
       no fast path) calls it once with round -1 and map == start_out == NULL, so that the
       ranks after it can fail at once instead of waiting for maps that never come.          */
    int (*carr_predict)(void *user, int round, const double *map, double *start_out);
} gss_run_opts_t;
int gss_run_ex(gss_dev *d, gss_scn *s, int64_t first_block, int64_t n_blocks, int batch,
               int threads, gss_sink_fn sink, void *user, const gss_run_opts_t *opts);


/* Exact carrier-chain helpers (exported for tests): advance the reference recurrence
   carr += step; wrap into [0,1) (gpssim.c:2245-2250) by n samples, exactly.                   */
double gss_carr_advance(double carr, double step, int64_t n);
/* Same over one block of n samples, also recording the GSS_NCK carrier checkpoints of the
   block (ck[j] = phase at sample (j*n)/GSS_NCK) for gss_synth_*'s carr_ck.  Returns the phase
   after the block, i.e. the next block's carr0.                                               */
double gss_carr_advance_ck(double carr, double step, int n, double *ck);
/* Same for the code phase with its chip/bit/word counters (gpssim.c:2212-2241).               */
double gss_code_advance(double code, double step, int64_t n, int32_t *icode, int32_t *ibit,
                        int32_t *iword);

/* The 512-entry carrier tables the sample loop uses (gpssim.c:15-83), generated.             */
int gss_lut(int32_t *sin512, int32_t *cos512);

const char *gss_last_error(void);
const char *gss_version(void);
/* Build configuration of the kernels, e.g. "lin_mfma=1 lin_ch=16 arch=gfx950" (lin_mfma: the fast
   path accumulates f16 x f16 products in f32 on the matrix cores, exact integer sums; 0: int64
   multiply-adds on the VALU).                                                                 */
const char *gss_build_info(void);

#ifdef __cplusplus
}
#endif
#endif /* GPSSIM_AMD_H */
