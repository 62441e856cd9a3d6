"""Device-resident rendering of a block range: the host plane (Scenario), the proofs
(gss_linearize_device on the GPU, or gss_linearize on the host) and gss_synth_lin_device in
batches, output left in HBM (a torch uint8 tensor).

Used by bench.py (timed steps over a resident window) and gpssim_amd.node (each rank renders its
time-window shard before the ordered gather to rank 0); the rows come from gpssim_amd.shard.  torch is only the allocator and stream
here; the kernels run through the C ABI.
"""
import time

import numpy as np

from . import (CHAN_DTYPE, LIN_DTYPE, MAXCH, NCK, block_bytes, ca_table, carr_advance_ck,
               linearize)


def block_checkpoints(blk, nch, n_per_blk, blocks=None):
    """the carrier checkpoints [nblk, 16, NCK] of the exact path's Stage A (gss_carr_advance_ck
    from each row's carr0), for `blocks` (default all); zeros elsewhere"""
    ck = np.zeros((len(nch), MAXCH, NCK), np.float64)
    for b in (range(len(nch)) if blocks is None else blocks):
        for k in range(int(nch[b])):
            ck[b, k] = carr_advance_ck(float(blk[b, k]["carr0"]), float(blk[b, k]["carr_step"]),
                                       n_per_blk)[1]
    return ck


class DeviceWindow:
    """One window of blocks, proven and resident in HBM, rendered in calls of at most `batch`
    blocks (each call's fast-path scratch rows scale with its block count), or in the calls
    `sizes` gives (block counts in row order: gpssim_amd.node's gather chunks)."""

    def __init__(self, torch, dev, dev_t, blk, nch, nav, n_per_blk, fmt, ck=None, threads=8,
                 batch=3000, out=None, proof="gpu", sizes=None):
        self.torch, self.dev, self.fmt, self.npb = torch, dev, fmt, n_per_blk

        def up(a):
            return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).to(dev_t)

        t0 = time.perf_counter()
        if proof == "gpu":                 # the proofs on the GPU: only the fast flags come back
            self.d_blk, self.d_nch = up(blk), up(np.asarray(nch, np.int32))
            ca = ca_table()
            self.d_ca, self.d_nav = up(ca), up(nav)
            nb = len(nch)
            self.d_lin = torch.empty(max(1, nb * MAXCH * LIN_DTYPE.itemsize), dtype=torch.uint8,
                                     device=dev_t)
            d_fast = torch.empty(max(1, nb), dtype=torch.int32, device=dev_t)
            stream = torch.cuda.current_stream(dev_t).cuda_stream
            if nb:
                dev.linearize_device(self.d_blk.data_ptr(), self.d_nch.data_ptr(), nb, n_per_blk,
                                     self.d_ca.data_ptr(), len(ca), self.d_nav.data_ptr(),
                                     len(nav), self.d_lin.data_ptr(), d_fast.data_ptr(), stream)
            fast = d_fast[:nb].cpu().numpy()           # (synchronises the stream)
            lin = None
        else:
            lin, fast = linearize(blk, nch, nav, n_per_blk, threads=threads)
        self.lin_s = time.perf_counter() - t0
        self.proof = proof
        self.nblk = len(nch)
        self.n_fast = int(fast.sum())
        # channel-samples the fast kernel renders per pass (its compute roofline's unit)
        self.ch_samples_fast = int(np.asarray(nch)[fast.astype(bool)].astype(np.int64).sum()) * \
            int(n_per_blk)
        self.nch_max = int(nch.max()) if len(nch) else 1
        ca = ca_table()
        self.n_ca, self.n_nav = len(ca), len(nav)
        self.bb = block_bytes(n_per_blk, fmt)

        if ck is None and self.n_fast < self.nblk:
            # rows planned without checkpoints (the chain run ahead, shard.plan_window): the
            # exact path's Stage A starts from them, so give the uncertified blocks theirs
            ck = block_checkpoints(blk, nch, n_per_blk, np.nonzero(fast == 0)[0])
        if lin is not None:
            self.d_blk, self.d_nch, self.d_lin = up(blk), up(nch), up(lin)
            self.d_ca, self.d_nav = up(ca), up(nav)
        self.d_ck = up(ck) if ck is not None else None
        self.d_fast = up(np.asarray(fast, np.int32))
        self.out = out if out is not None else torch.empty(self.nblk * self.bb, dtype=torch.uint8,
                                                           device=dev_t)
        assert self.out.numel() >= self.nblk * self.bb
        self.batches = []
        if sizes is None:
            sizes = [min(batch, self.nblk - b0) for b0 in range(0, self.nblk, batch)]
        assert sum(sizes) == self.nblk and all(n > 0 for n in sizes)
        b1 = 0
        for n in sizes:
            b0, b1 = b1, b1 + n
            fb = np.nonzero(fast[b0:b1] == 0)[0].astype(np.int32)
            d_fb = torch.from_numpy(fb if len(fb) else np.zeros(1, np.int32)).to(dev_t)
            self.batches.append((b0, b1, d_fb, len(fb)))
        if self.nblk:
            dev.reserve(max(sizes), n_per_blk)

    def step(self, stream=0, lin=None, fast=None):
        """Render every block of the window into self.out (stream-ordered).  lin, fast: device
        tensors holding the window's certified lines and fast flags in place of d_lin, d_fast
        (a second set proven while this one renders: bench.py's device_pipeline)."""
        for i in range(len(self.batches)):
            self.step_batch(i, stream, lin, fast)

    def step_batch(self, i, stream=0, lin=None, fast=None):
        """Render batch i (blocks batches[i][0] .. batches[i][1]) into its part of self.out."""
        cs, ls, ks = CHAN_DTYPE.itemsize * MAXCH, LIN_DTYPE.itemsize * MAXCH, 8 * MAXCH * NCK
        d_lin = self.d_lin if lin is None else lin
        d_fast = self.d_fast if fast is None else fast
        for b0, b1, d_fb, n_fb in self.batches[i:i + 1]:
            self.dev.synth_lin_device(
                self.d_blk.data_ptr() + b0 * cs, self.d_nch.data_ptr() + b0 * 4, self.nch_max,
                d_lin.data_ptr() + b0 * ls, d_fast.data_ptr() + b0 * 4,
                d_fb.data_ptr(), n_fb, self.d_ca.data_ptr(), self.n_ca, self.d_nav.data_ptr(),
                self.n_nav, b1 - b0, self.npb, self.fmt, self.out.data_ptr() + b0 * self.bb,
                stream=stream,
                ck_ptr=(self.d_ck.data_ptr() + b0 * ks) if self.d_ck is not None else 0)

    def free_inputs(self):
        for a in ("d_blk", "d_nch", "d_lin", "d_ck", "d_ca", "d_nav", "d_fast"):
            setattr(self, a, None)
        self.batches = []

    def free(self, release=True):
        """Drop the window's buffers; release=False keeps them in torch's cache instead of
        returning them to the driver, which wipes released device memory with the copy engines
        in the background and so slows this process's device -> host copies for a while
        (tools/e2e_bench_probe.py)."""
        self.free_inputs()
        self.out = None
        if release:
            self.torch.cuda.empty_cache()
