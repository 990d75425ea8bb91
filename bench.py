"""BICOS hot-path benchmark (driver contract: one JSON line on rank 0).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2]
  torchrun --nproc-per-node N bench.py --gpus N ...      (one process per GPU, RCCL)

A step = one full BICOS::match of the configured synthetic stereo frame
(transform x2 -> Hamming search -> NXC agree [-> subpixel]) with the planar
stacks already resident in HBM. With N > 1 the frame is split into N row bands
(one per GPU, strong scaling) and the disparity + correlation bands are gathered
to rank 0 with ONE RCCL gather per step, inside the timed region; the gather of
step k overlaps the kernels of step k+1 (double-buffered), and every gather has
completed before the closing barrier.

Frames in flight (--inflight F; on one GPU per config -- 1 for cfg2 / cfg5, 2 for
cfg1 / cfg3 / cfg4 / readme / integ-* -- and 6 for row bands on N > 1): step k runs on stream k % F with its own
engine and output buffers, so consecutive frames overlap the way a camera stream is
processed -- the HBM-bound transform / agree of one frame fill the compute-unit slots the
previous frame's search leaves idle in its last round of workgroups (narrow row bands:
192 rows at N = 8). Every step still does the whole match into its own buffers; `value`
and `ms_per_step` are the throughput over the K steps, and `ms_per_match_one_at_a_time`
is the latency of one match with nothing overlapping it (this rank's band, no gather).

Extra keys on the JSON line:
  roofline      the dominant kernel (the Hamming search), timed live with HIP
                events on the stream it runs on. Default (matrix-core search,
                search_mx.hip): algorithmic FP4 MFMA FLOPs per launch (2 x descriptor
                bits per Hamming pair) / average launch time vs the dense FP4 MFMA
                peak; `valu_view` holds the key-reduction issue bound that actually
                binds it. BICOS_SEARCH=valu: pairs/s vs the VALU
                issue bound of the popcount search. `hbm` holds the HBM-bound stages
                (transform, agree) against the 8 TB/s peak.
  cpu_baseline  the C oracle (oracle/bicos_oracle.c, -march=x86-64-v3; the as-shipped
                -O3 build beside it) on every host core this process may use, rank 0
                at N=1 only, over a bounded row sample (CPU model / nproc stated).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# MI355X (gfx950) peaks. HBM: /opt/skills/guides/MI355X_MICROARCH.md "Chip-level
# parameters" (8 TB/s). VALU: the guide gives no integer rates, so they were measured on
# the box (tools/valu_peak.hip -> profiles/valu_rates_r01.json): v_xor/v_and/v_add/v_mov
# issue at full rate, ~72 T lane-op/s (128 lanes/clk/CU at the held clock); v_bcnt,
# v_min/med3, v_lshl_or, v_perm, v_pk_*_u16 at half rate, ~38.5 T lane-op/s.
HBM_PEAK_GBS = 8000.0
VALU_FULL_TOPS = 72.0
VALU_HALF_TOPS = 38.5
VALU_NOMINAL_TOPS = 256 * 128 * 2.4e9 / 1e12   # 78.6: every op at full rate, 2.4 GHz
# Dense FP4 MFMA peak (MI355X_MICROARCH.md "Peak FP6/FP4 MFMA": ~10 PF dense, the 20 PF
# figure is 2:1 sparsity): v_mfma_scale_f32_32x32x64_f8f6f4 on FP4 operands.
MFMA_FP4_DENSE_TFLOPS = 10000.0
# sustained v_mfma_scale_f32_32x32x64_f8f6f4 (FP4) rate measured on the box, 4 waves/SIMD
# (tools/mfma_rate.hip, profiles/mfma_rates_r01.jsonl): the clock the pipe actually runs at
MFMA_FP4_SUSTAINED_TFLOPS = 8360.0

CONFIGS = {
    # BASELINE.json configs; "cfg2" is the one the headline metric is quoted on
    "cfg1": dict(n=8, H=480, W=640, dtype="u8", cfg=dict(nxcorr_threshold=0.9),
                 desc="8x2 stack @ 640x480 u8, LIMITED 32-bit, nxcorr 0.9"),
    "cfg2": dict(n=33, H=1536, W=2048, dtype="u8", cfg=dict(nxcorr_threshold=0.96),
                 desc="33x2 stack @ 2048x1536 u8, LIMITED 128-bit (4n-7=125 bits), nxcorr 0.96"),
    "cfg3": dict(n=33, H=1536, W=2048, dtype="u8",
                 cfg=dict(nxcorr_threshold=0.96, min_variance=2.0, subpixel_step=0.1),
                 desc="33x2 @ 2048x1536 u8, 128-bit, nxcorr 0.96, min-variance 2.0, subpixel 0.1"),
    "cfg4": dict(n=40, H=1536, W=2048, dtype="u8",
                 cfg=dict(nxcorr_threshold=0.96, variant=1, max_lr_diff=1),
                 desc="40x2 @ 2048x1536 u8, LIMITED 256-bit, LR-consistency max_lr_diff 1, nxcorr 0.96"),
    "cfg4f": dict(n=40, H=1536, W=2048, dtype="u8", cfg=dict(nxcorr_threshold=0.96),
                  desc="40x2 @ 2048x1536 u8, LIMITED 256-bit, NoDuplicates, nxcorr 0.96 (cfg4 "
                       "without Consistency; not a BASELINE config)"),
    "cfg5": dict(n=33, H=2160, W=3840, dtype="u8", cfg=dict(nxcorr_threshold=0.96),
                 desc="33x2 @ 3840x2160 u8, 128-bit, nxcorr 0.96"),
    # the reference README's published full match (README.md:80,90: ~44 ms on an RTX 4090,
    # dataset 3208x2200 per example-disp.png): bicos-cli --limited --threshold 0.96
    # --stacksize 33 --variance 2.0 --step 0.1
    "readme": dict(n=33, H=2200, W=3208, dtype="u8",
                   cfg=dict(nxcorr_threshold=0.96, min_variance=2.0, subpixel_step=0.1),
                   desc="33x2 @ 3208x2200 u8, LIMITED 128-bit, nxcorr 0.96, min-variance 2.0, "
                        "subpixel 0.1 (reference README.md:80,90 full match)",
                   published={"ms_per_match": 44.0, "hardware": "RTX 4090",
                              "source": "reference README.md:90 (~44 ms)"}),
}

# The reference's integration bench (bench/cuda.cu:297-323, grid :397-401): cuda::match in
# FULL mode, nxcorr threshold 0.9, n = 6/8/12/16 images x subpixel step none / 0.25 / 0.20 /
# 0.15 / 0.10, one match at a time, on its dataset (3208x2200 per README example-disp.png;
# the dataset is download-only, so the frame here is the synthetic planted-disparity one).
# Published RTX 4090 times: bench/baselines/cuda-rtx4090.txt:67-86.
INTEG_RTX4090_MS = {
    (6, 0): 11.020829, (8, 0): 14.068066, (12, 0): 24.826253, (16, 0): 52.028470,
    (6, 25): 11.721331, (8, 25): 15.127557, (12, 25): 26.694482, (16, 25): 55.497395,
    (6, 20): 11.770639, (8, 20): 15.202322, (12, 20): 26.801793, (16, 20): 55.480473,
    (6, 15): 11.940925, (8, 15): 15.211238, (12, 15): 26.902525, (16, 15): 56.758473,
    (6, 10): 12.146678, (8, 10): 15.711815, (12, 10): 27.856642, (16, 10): 57.357942,
}
for (_n, _s), _ms in INTEG_RTX4090_MS.items():
    _cfg = dict(nxcorr_threshold=0.9, mode=1)
    if _s:
        _cfg["subpixel_step"] = _s / 100.0
    CONFIGS["integ-n%d%s" % (_n, "-s%d" % _s if _s else "")] = dict(
        n=_n, H=2200, W=3208, dtype="u8", cfg=_cfg,
        desc="%dx2 @ 3208x2200 u8, FULL %d-bit, nxcorr 0.9%s (reference integration bench, "
             "bench/cuda.cu:297-323)" % (_n, 32 * (1 if _n * _n - 2 * _n + 3 <= 32 else
                                                   2 if _n * _n - 2 * _n + 3 <= 64 else
                                                   4 if _n * _n - 2 * _n + 3 <= 128 else 8),
                                          ", subpixel %.2f" % (_s / 100.0) if _s else ""),
        published={"ms_per_match": _ms, "hardware": "RTX 4090", "timing": "one match at a time",
                   "source": "reference bench/baselines/cuda-rtx4090.txt:67-86 "
                             "(bench_integration/%d/%d)" % (_n, _s)})
del _n, _s, _ms, _cfg


# Frames in flight at N = 1, per config: F = 1 / 2 / 3 interleaved twice in
# one session at the driver's 20 steps and at 200 (profiles/inflight_r06.jsonl). A config
# keeps 2 only where 2 won by more than the run-to-run spread (~1.3 %): cfg1 (launch-bound:
# 13030 vs 9729 Mpix/s at F = 1), cfg3 (the subpixel refine overlaps the next frame's search:
# +2.6 %), readme (+1.9 %) and the integration grid (FULL n = 6 / 8 / 12 / 16 +5.9 / +2.7 /
# +1.3 / +1.5 %, n = 12 with subpixel +2.2 %). cfg2 / cfg5: F = 1 (cfg2 7740 vs 7668 at 20
# steps, 7751 vs 7824 at 200; cfg5 4741 vs 4693). cfg4 with the one-launch Consistency search
# (re-measured): F = 2, 4288 / 4316 vs 4270 / 4267 at 20 steps, 4368 / 4363 vs 4260 / 4278 at 200.
INFLIGHT_DEFAULT = {"cfg1": 2, "cfg3": 2, "cfg4": 2, "readme": 2}


def inflight_default(config: str) -> int:
    if config.startswith("integ-"):
        return 2
    return INFLIGHT_DEFAULT.get(config, 1)


def search_pairs(rows: int, W: int, cfg: dict) -> float:
    """Hamming pairs of one pass over the cost matrix: every (col0, col1) of every row.
    Consistency searches it twice (forward, then the full reverse; callers double it)."""
    return float(rows) * W * W


def search_pair_peak(words: int, cfg: dict) -> float:
    """Issue-rate bound in pairs/s of the VALU search's per-pair instruction mix at the
    measured VALU rates (search16_kernel): `words` v_xor (full rate) + `words` v_bcnt (half
    rate) + half a v_perm and half a v_pk_min_u16 (2 col0 share one packed key register) +
    with duplicate detection another half v_xor (full) and half v_pk_min_u16 (half)."""
    dupes = cfg.get("variant", 0) == 0 or cfg.get("no_dupes", False)
    full = words + (0.5 if dupes else 0.0)
    half = words + 1.0 + (0.5 if dupes else 0.0)
    per_pair_s = full / (VALU_FULL_TOPS * 1e12) + half / (VALU_HALF_TOPS * 1e12)
    return 1.0 / per_pair_s


def search_ops(rows: int, W: int, words: int, cfg: dict) -> float:
    """INT32 lane-ops of one pass over the cost matrix with 32-bit keys: per pair `words`
    xor + `words` bcnt + key pack + min (+ med3 with NoDuplicates) = 2w+3 (2w+2 without)."""
    dupes = cfg.get("variant", 0) == 0 or cfg.get("no_dupes", False)
    return search_pairs(rows, W, cfg) * (2 * words + (3 if dupes else 2))


def subpixel_steps(step: float) -> int:
    """x values of the reference's refine loop, for (float x = -1; x <= 1; x += step)
    accumulated in float32 (agree.hpp:122; engine.cpp subpixel_steps)."""
    import numpy as np
    x, k, st = np.float32(-1.0), 0, np.float32(step)
    while x <= np.float32(1.0):
        k += 1
        x = np.float32(x + st)
    return k


def mx_search() -> bool:
    """The pipeline's search runs on the matrix cores unless BICOS_SEARCH=valu
    (engine.cpp use_mx)."""
    return os.environ.get("BICOS_SEARCH", "") != "valu"


def mx_ksteps(words: int, bits: int) -> int:
    """64-bit K-steps the matrix-core search multiplies (search_mx.hip
    search_mx_geometry): all of the descriptor, except 3 of 4 for 256-bit descriptors
    whose used bits (the transform's 4n-5 / n^2-2n+3) fit in 192."""
    ks = max(1, words // 2)
    if words == 8 and 0 < bits <= 192:
        ks = 3
    return ks


def mx_flops(rows: int, W: int, words: int, cfg: dict, bits: int = 0, set_bits: int = 0,
             reverse_col1: float | None = None):
    """(algorithmic, used-bit) FLOPs of the matrix-core search per launch. Each Hamming pair
    is a K-long dot product (2K FLOPs). Algorithmic K = the descriptor bits the kernel
    multiplies: the descriptor type's width (128 for u128, the reference's popcount width),
    or fewer when whole 64-bit K-steps above the used bits are skipped (cfg4: 192 of 256;
    mx_ksteps) -- never more than executed. Used-bit K = the bits the transform actually
    sets (4n-6 LIMITED: 126 at n = 33, 154 at n = 40), the stricter view. Consistency runs
    the forward search and the reverse search over the `reverse_col1` distinct col1 the
    forward search kept (engine.cpp reverse_search; every col1 when None)."""
    pairs = search_pairs(rows, W, cfg)
    if cfg.get("variant", 0) == 1:
        pairs += float(reverse_col1 if reverse_col1 is not None else rows * W) * W
    k_exec = min(32 * words, 64 * mx_ksteps(words, bits))
    k_used = min(k_exec, set_bits) if set_bits else k_exec
    return pairs * 2 * k_exec, pairs * 2 * k_used


def transform_bits(n: int, mode: int) -> int:
    """Descriptor bits the transform sets: LIMITED 4n-6 (n >= 4; 7 / 4 for n = 3 / 2), FULL
    n^2-2n+3 (descriptor_transform.hpp:31-123; tests/test_oracle.py pins both)."""
    if mode:
        return n * n - 2 * n + 3
    return 4 * n - 6 if n >= 4 else (7 if n == 3 else 4)


def pk_key_pair_peak() -> float:
    """Issue bound in pairs/s of the packed-key search's VALU key reduction (search_mx.hip
    search_pk_kernel) at the measured rates. Per wide tile (64 col0) and block (32 col1),
    2048 pairs, every lane issues the pk_tree (7 v_pk_minimum3_f16 + 1 v_pk_min_u16) and its
    share of the pair step (v_permlane32_swap, v_pk_min_u16, v_pk_sub_u16, v_pk_min_u16 per
    two tiles: 2 half-rate ops per tile) -- 10 half-rate instructions -- plus the tie / drop
    test (v_and + v_cmp per two tiles: 1 full-rate); the rare new-minimum branch is not
    counted. Per pair: 10 x 64 / 2048 half-rate and 64 / 2048 full-rate lane-ops."""
    half = 10.0 * 64 / 2048
    full = 1.0 * 64 / 2048
    return 1.0 / (full / (VALU_FULL_TOPS * 1e12) + half / (VALU_HALF_TOPS * 1e12))


# Fraction of (tile, block) units of the NoDuplicates search that take the last-minimum
# branch on the planted-disparity frames: ~5.6 reaching blocks per tile and row scan whatever
# the width (tools/reach_sim.py: 2048 columns 0.068 / 0.094 / 0.103 at rows 0 / 767 / 1535,
# 3840 columns 0.047), i.e. ~180 / cols; random descriptors reach on ~0.73.
def mx_reach_planted(cols: int) -> float:
    return min(1.0, 180.0 / max(cols, 1))


MX_REACH_PLANTED = mx_reach_planted(2048)


def mx_key_pair_peak(words: int, cfg: dict, reach: float = MX_REACH_PLANTED) -> float:
    """Issue bound in pairs/s of the matrix-core search's VALU key reduction AS EXECUTED, at
    the measured rates: the instructions per (wave, 32-col0 tile, 32-col1 block) = 1024 pairs
    of the ISA of search_mx_kernel (DESIGN.md s5.1 audit). NoDuplicates (KEYS 2): every unit
    8 v_min3_u32 (half rate, the first-minimum tree) + 3.5 full-rate (its share of the
    pair step: v_permlane32_swap, 2 v_min_u32, v_add, v_or, v_cmp per two tiles; the
    prefetch address per four); a unit that reaches the running minimum (fraction `reach`)
    adds the last-minimum tree: 16 v_xor + 2 integer (full) and 8 v_min3 (half). First
    minimum only (Consistency without NoDuplicates, FK / XK keys): 8 v_min3 (half) + 1 full
    (the frame shift). (Round 5 counted the last-minimum tree on every pair: 1 full + 1 half
    lane-op per pair, an upper bound 2.1x the executed count at cfg2.)"""
    dupes = cfg.get("variant", 0) == 0 or cfg.get("no_dupes", False)
    if dupes:
        half, full = 8.0 + 8.0 * reach, 3.5 + 18.0 * reach
    else:
        half, full = 8.0, 1.0
    per_unit_s = half * 64 / (VALU_HALF_TOPS * 1e12) + full * 64 / (VALU_FULL_TOPS * 1e12)
    return 1024.0 / per_unit_s


def lr_key_pair_peak(tiles: int = 4) -> float:
    """Issue bound in pairs/s of the one-pass Consistency search's VALU (search_mx.hip
    search_lr_kernel), from its ISA per wave and block of `tiles` x 32 col0 x
    32 col1 pairs: forward 8 v_min3_f32 (half rate) + 1 v_sub_f32 per tile; the reverse keys'
    minimum over the tiles (16 v_min_u32, then 16 v_min3_u32 per further pair: half); the lane
    transposition (8 v_permlane16_swap at a quarter rate, 8 + 7 DPP + 1 v_min_u32: half; 14
    v_cndmask, a v_mov_dpp, a v_add_f32: full) and ~6 address / exec VALU (full). T = 4 (the
    default): 96 half-rate and 26 full-rate instructions per 4096 pairs; T = 2 (BICOS_LR_T=2):
    56 and 22 per 2048."""
    if tiles == 2:
        half, full, pairs = 56.0, 22.0, 2048.0
    else:
        half, full, pairs = 96.0, 26.0, 4096.0
    per_pair_s = half * 64 / pairs / (VALU_HALF_TOPS * 1e12) + full * 64 / pairs / (VALU_FULL_TOPS * 1e12)
    return 1.0 / per_pair_s


def mx_key_pair_peak_all_trees() -> float:
    """The round-5 key-reduction model (both trees on every pair: 1 v_xor + 1 v_min3 per
    pair), kept as the upper-bound view VERDICT r05 quoted (25.1 Tpairs/s)."""
    return 1.0 / (1.0 / (VALU_FULL_TOPS * 1e12) + 1.0 / (VALU_HALF_TOPS * 1e12))


def kernel_source_hash() -> str:
    """sha256 over the HIP kernel and host sources of libbicos_amd.so (csrc/, sorted). The PMC
    summaries record it (tools/pmc_summary.py), and a bench line cites their HBM bytes only
    when they were measured on the very sources it runs."""
    import glob
    import hashlib
    h = hashlib.sha256()
    for f in sorted(glob.glob(os.path.join(ROOT, "libbicos_amd", "csrc", "*"))):
        if f.rsplit(".", 1)[-1] in ("hip", "hpp", "cpp", "h") or f.endswith("Makefile"):
            h.update(os.path.basename(f).encode())
            h.update(open(f, "rb").read())
    return h.hexdigest()[:16]


def load_traffic(kernel_prefix, config: str, rows: int):
    """HBM bytes per frame (PMC FETCH_SIZE x2 + WRITE_SIZE, gfx950 corrections) of the kernels
    whose names start with `kernel_prefix` (a string or a tuple of them) from the committed
    profiles/pmc_r*.json entries for this config and row count, measured on the current
    sources (kernel_source_hash). A stage can be several dispatches per frame -- Consistency's
    forward and reverse search, a search's tail launch (search_mx.hip launch_mx_tt) -- so each
    kernel group's per-dispatch bytes count as often as it was dispatched per frame (frames =
    the fewest dispatches of any kernel of the config). Returns {"bytes", "source"}, or
    {"bytes": None, "why": ...} when no such profile exists."""
    import glob
    prefixes = (kernel_prefix,) if isinstance(kernel_prefix, str) else tuple(kernel_prefix)
    want = kernel_source_hash()
    stale = None
    for f in reversed(sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_r*.json")))):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        mine = [(key, c) for key, c in d.get("kernels", {}).items()
                if c.get("config") == config and c.get("rows") == rows and
                "hbm_read_bytes" in c and "hbm_write_bytes" in c]
        hits = [(key, c) for key, c in mine if c.get("kernel", "").startswith(prefixes)]
        if not hits:
            continue
        src = os.path.relpath(f, ROOT) + " :: " + "; ".join(key for key, _ in hits)
        if d.get("source_sha") != want:
            stale = stale or src
            continue
        frames = min(int(c.get("dispatches", 1)) for _, c in mine) or 1
        rd = sum(c["hbm_read_bytes"] * int(c.get("dispatches", frames)) for _, c in hits) / frames
        wr = sum(c["hbm_write_bytes"] * int(c.get("dispatches", frames)) for _, c in hits) / frames
        return {"bytes": rd + wr, "read_bytes": rd, "write_bytes": wr, "source": src,
                "source_sha": want}
    return {"bytes": None, "why": ("PMC profile %s was taken on other sources" % stale) if stale
            else "no PMC profile for %s rows=%d" % (config, rows), "source_sha": want}


def launch_ranks(world: int) -> int:
    """One child process per rank (what torchrun would start): RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_ADDR=127.0.0.1 / a free MASTER_PORT in the environment, the same
    argv. Rank 0 prints the JSON line (the children share our stdout); the other ranks print
    nothing. Returns the first non-zero exit status, else 0. A rank that fails takes the
    others down (they would block in the next collective)."""
    import signal
    import socket
    import subprocess

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world),
                   LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                for q in live:
                    q.send_signal(signal.SIGTERM)
        if live:
            time.sleep(0.05)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--spinup-ms", type=float, default=100.0,
                    help="untimed warm-up lasts at least this long (GPU clock ramp), >= W steps")
    ap.add_argument("--config", default="cfg2", choices=sorted(CONFIGS))
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                    help="strong: one frame split in row bands; weak: a full frame per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="target wall time of the CPU baseline sample")
    ap.add_argument("--kernel-reps", type=int, default=10)
    ap.add_argument("--inflight", type=int, default=None,
                    help="frames in flight: step k runs on stream k %% F with its own engine, so "
                         "one frame's HBM-bound stages fill the slots the previous frame's "
                         "search leaves idle (1 = strictly one match after another). Default on "
                         "one GPU: per config (INFLIGHT_DEFAULT: 2 for cfg1 / cfg3 / cfg4 / readme / the "
                         "integration grid, else 1; "
                         "profiles/inflight_r06.jsonl), 6 for N > 1 row bands and --band-of "
                         "(band 0 of 8: cfg5 0.2140-0.2146 vs 0.2244-0.2281 ms with 3, cfg2 within "
                         "1 %%; profiles/bands_inflight_r05.jsonl)")
    ap.add_argument("--no-host-path", action="store_true",
                    help="skip the end-to-end host-buffer measurement (rank 0, N=1)")
    ap.add_argument("--selftest-launch", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (production); gloo = rehearsal of the N>1 "
                         "path with several ranks sharing one GPU (not a measurement)")
    ap.add_argument("--verify-gather", action="store_true",
                    help="(default; kept for old command lines) verify the gathered frames")
    ap.add_argument("--no-verify-gather", action="store_true",
                    help="skip the untimed check of the gathered frames (by default, after the "
                         "timed run, NB more steps land over a sentinel and rank 0 checks every "
                         "gather slot's whole frame against the oracle's sha256 in "
                         "tests/golden/frames.json, or a one-GPU match of the whole frame)")
    ap.add_argument("--gather-rehearsal", action="store_true",
                    help="one rank, and still the whole N>1 gather path on a 1-rank process group "
                         "(--backend nccl: RCCL init, the packed band buffer gathered from the "
                         "match's streams, the int16 landing, the gather timing and the frame "
                         "verification) -- rehearses the RCCL branch on a one-GPU box (not a "
                         "measurement)")
    ap.add_argument("--gather", default="auto", choices=["auto", "dma", "rccl"],
                    help="N > 1: how the bands reach rank 0. rccl: one RCCL gather per step (its "
                         "receive runs on rank 0's compute units, beside rank 0's own band: "
                         "profiles/root_gather_r05.jsonl); dma: every rank copies its band "
                         "straight into rank 0's receive slot (IPC-mapped) with hipMemcpyAsync on "
                         "its own stream -- the copy engines of the sending GPU, nothing on rank "
                         "0's CUs -- and a one-element RCCL all_reduce per step orders the frame; "
                         "auto (default): dma when its setup self-test passes on every rank, else "
                         "rccl")
    ap.add_argument("--band-of", type=int, default=1,
                    help="one process, band 0 of an N-way row split (no gather): the band a "
                         "rank of an N-GPU run computes, for profiling at band sizes")
    ap.add_argument("--root-load", default=None, choices=["kernel", "proxy", "dma"],
                    help="with --band-of N: rehearse rank 0's gather ingress on one GPU -- per "
                         "step, on a side stream, the N-1 other bands' packed maps are written "
                         "into a root buffer: by a full-grid torch copy kernel (kernel), by "
                         "--root-load-wgs long-lived copy workgroups the way RCCL receives on the "
                         "root's CUs (proxy: tools/ingress_proxy.hip), or by the copy engines (dma: "
                         "hipMemcpyAsync kind hipMemcpyDeviceToDeviceNoCU from a second HBM buffer, "
                         "split over --root-load-streams streams). Every form lands every step's "
                         "bytes, with the gather pipeline's back pressure. Reports the band's rate "
                         "under that load and the achieved ingress.")
    ap.add_argument("--root-load-streams", type=int, default=2,
                    help="--root-load dma: side streams the per-step copy is split over (1-4)")
    ap.add_argument("--root-load-wgs", type=int, default=16,
                    help="--root-load proxy: copy workgroups (RCCL channels x peers)")
    ap.add_argument("--root-load-high-priority", action="store_true",
                    help="--root-load: the ingress stream at high priority")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `python bench.py --gpus N` without torchrun: start the N ranks ourselves, before
        # this process touches torch or HIP (no exec from a GPU-initialised process)
        raise SystemExit(launch_ranks(args.gpus))

    import numpy as np
    import torch
    import torch.distributed as dist

    if args.selftest_launch:
        # launcher check without a GPU (tests/test_bench_launch.py): the ranks rendezvous
        # over gloo exactly as the bench does and rank 0 reports what it saw
        world = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        if os.environ.get("BICOS_SELFTEST_FAIL_RANK") == str(rank):
            raise SystemExit(3)
        if world > 1:
            dist.init_process_group("gloo")
        t = torch.tensor([rank + 1.0])
        if world > 1:
            dist.all_reduce(t)
        if rank == 0:
            print(json.dumps({"selftest": "launch", "world": world, "gpus": args.gpus,
                              "rank_sum": float(t.item()),
                              "pid_parent": os.getppid()}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    from libbicos_amd import _lib, device
    from libbicos_amd.distributed import band_height, band_rows
    from libbicos_amd.synthetic import stereo_stack

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE=%d (launch N>1 with torchrun)" % (args.gpus, world))
    ndev = torch.cuda.device_count()
    if args.backend == "nccl" and local >= ndev:
        raise SystemExit("rank %d has no GPU (%d visible)" % (local, ndev))
    local_dev = local % ndev
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    if args.gather_rehearsal and world != 1:
        raise SystemExit("--gather-rehearsal runs one rank")
    # a process group whenever the gather path runs (N > 1, or the 1-rank rehearsal)
    dist_on = world > 1 or args.gather_rehearsal
    if dist_on:
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if "MASTER_PORT" not in os.environ:
                import socket
                with socket.socket() as so:
                    so.bind(("127.0.0.1", 0))
                    os.environ["MASTER_PORT"] = str(so.getsockname()[1])
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, rank=rank, world_size=world)
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)

    C = CONFIGS[args.config]
    n, H, W = C["n"], C["H"], C["W"]
    mcfg = device.MatchConfig(**C["cfg"])
    words = device.descriptor_words(n, mcfg.mode)
    if args.scaling == "strong":
        b, e = band_rows(H, world, rank)
    else:
        b, e = 0, H
    if args.band_of > 1:
        if world != 1:
            raise SystemExit("--band-of is a one-process profiling mode")
        b, e = band_rows(H, args.band_of, 0)
    rows = e - b

    # synthetic stacks of this rank's band, generated on the host once, resident in HBM
    L, R = stereo_stack(n, H, W, np.uint8, row_begin=b, row_end=e)
    s0 = torch.from_numpy(L).to(dev)
    s1 = torch.from_numpy(R).to(dev)
    del L, R
    F = max(1, args.inflight if args.inflight is not None else
            (inflight_default(args.config) if world == 1 and args.band_of == 1 else 6))
    # one engine (workspace) and one stream per frame in flight; slot 0 = torch's stream
    engines = [device.Engine(local_dev) for _ in range(F)]
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(F - 1)]
    eng = engines[0]
    has_corr = mcfg.nxcorr_threshold is not None
    outs = [torch.empty((rows, W), dtype=torch.float32 if has_corr else torch.int16, device=dev)
            for _ in range(F)]
    corrs = [torch.empty((rows, W), dtype=torch.float32, device=dev) if has_corr else None
             for _ in range(F)]
    out, corr = outs[0], corrs[0]

    gather = dist_on and args.scaling == "strong"
    nccl = args.backend == "nccl"
    # integer disparities (NXC without subpixel): the band ships its disparity as int16 --
    # (float) of it IS the float map -- and rank 0 converts the gathered frame back to float32
    # with one op: 6 instead of 8 bytes per pixel over xGMI
    i16 = has_corr and mcfg.subpixel_step is None
    if gather:
        hb = band_height(H, world)
        # one packed [disparity | corrmap] band buffer (bytes) -> ONE RCCL gather per step.
        # The match writes straight into it (no copies); the buffers alternate (at least two,
        # one per frame in flight) so step k's gather (RCCL stream) overlaps later steps'
        # kernels.
        dbytes = hb * W * (4 if has_corr and not i16 else 2)  # float map only with subpixel
        off = (dbytes + 3) // 4 * 4
        nbytes = off + (hb * W * 4 if has_corr else 0)
        # dma: the band buffers live on the GPU even for a gloo rehearsal (ranks sharing one
        # GPU); decided with a self-test below (auto), before anything is timed
        want_dma = args.gather in ("auto", "dma") and world > 1
        gdev = dev if (nccl or want_dma) else torch.device("cpu")
        # dma: a slot is rewritten only after the frame two steps back is complete (lag L =
        # 2), so 2L slots keep every write behind the landing of the frame it replaces
        NB = max(4, F) if want_dma else max(2, F)
        sends = [torch.zeros(nbytes, dtype=torch.uint8, device=gdev) for _ in range(NB)]
        recv_all = [torch.empty((world, nbytes), dtype=torch.uint8, device=gdev) if rank == 0
                    else None for _ in range(NB)]
        recvs = [list(r.unbind(0)) if r is not None else None for r in recv_all]
        pending = [None] * NB
        dma = setup_dma_gather(args, dist, torch, dev, nccl, rank, world, recv_all, sends,
                               nbytes) if want_dma else None
        if dma is None and want_dma and not nccl:
            # (the rccl-form rehearsal over gloo moves host buffers)
            raise SystemExit("--gather dma setup failed on a gloo rehearsal")
        gather_choice = None
        if dma is not None and nccl and args.gather == "auto":
            # auto (round 6): both gathers timed alone before anything is timed; the
            # copy-engine one is kept unless it is slower than 1.25 x the RCCL gather. One GPU
            # cannot rehearse it at rate (profiles/root_gather_r06.jsonl: HBM-to-HBM copy
            # engines reach 34-135 GB/s of the 50-301 GB/s rank 0 needs), and
            # its advantage -- nothing on rank 0's compute units -- is worth a slower transfer
            # only up to a point
            t_dma = time_dma_exchange(dist, torch, dev, rank, world, dma, streams[0], nbytes, reps=5)
            t_rccl = time_gather(dist, torch, dev, nccl, rank, sends[0], recvs[0], nbytes, world,
                                 reps=5)
            tt = torch.tensor([t_rccl["ms"]], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            ms_rccl = float(tt.item())
            keep = t_dma["ms_per_exchange"] <= 1.25 * ms_rccl
            gather_choice = {"dma_ms_per_exchange": t_dma["ms_per_exchange"],
                             "rccl_ms_per_gather": round(ms_rccl, 4),
                             "rule": "dma unless its exchange takes > 1.25 x the RCCL gather",
                             "chosen": "dma" if keep else "rccl"}
            if not keep:
                dma = None
        # rank 0: the float32 disparity frame of each gather slot (one per slot,
        # so a stale or misordered landing cannot hide behind a shared buffer)
        frame_disps = [torch.empty((world, hb, W), dtype=torch.float32, device=gdev)
                       for _ in range(NB)] if rank == 0 and i16 else None

        def disp_view(buf):  # [hb, W] disparity plane of a packed buffer (or [world, hb, W])
            d = buf[..., :dbytes].view(torch.int16 if i16 else
                                       (torch.float32 if has_corr else torch.int16))
            return d.view(buf.shape[:-1] + (hb, W))

        def corr_view(buf):
            return buf[..., off:].view(torch.float32).view(buf.shape[:-1] + (hb, W))

        def land(i):  # rank 0, gather i complete: the frame's float disparity map
            pending[i].wait()
            pending[i] = None
            if rank == 0 and i16:
                frame_disps[i].copy_(disp_view(recv_all[i]))

        def dma_step(k, f):
            # lag 2: the frame of step k-2 is complete everywhere before step k writes (rank 0
            # lands it first); see setup_dma_gather for why every write is then safe
            i = k % NB
            j = k - 2
            if j >= 0 and pending[j % NB] is not None:
                land(j % NB)
            if rank == 0:
                engines[f].match(s0, s1, mcfg, out=disp_view(recv_all[i][0])[:rows],
                                 corrmap=corr_view(recv_all[i][0])[:rows] if has_corr else None)
            else:
                buf = sends[i]
                engines[f].match(s0, s1, mcfg, out=disp_view(buf)[:rows],
                                 corrmap=corr_view(buf)[:rows] if has_corr else None)
                dma["copy"](i, streams[f])
            pending[i] = dma["signal"](i, streams[f])
    state = {"k": 0}

    # --root-load: the bytes rank 0 of an N-way run receives per step (the other bands'
    # packed [disparity | corrmap] buffers: 6 B/px with int16 disparities, 8 with subpixel)
    load = None
    if args.root_load:
        if args.band_of < 2 or world != 1:
            raise SystemExit("--root-load rehearses rank 0 of --band-of N (one process)")
        bpp = (2 if (i16 or not has_corr) else 4) + (4 if has_corr else 0)
        ing = (args.band_of - 1) * band_height(H, args.band_of) * W * bpp
        ing = (ing + 15) // 16 * 16
        nst = max(1, min(4, args.root_load_streams)) if args.root_load == "dma" else 1
        load = {"mode": args.root_load, "bytes_per_step": ing, "issued": 0, "skipped": 0,
                "dst": torch.empty(ing // 4, dtype=torch.int32, device=dev),
                "src": torch.ones(ing // 4, dtype=torch.int32, device=dev),
                "stream": torch.cuda.Stream(dev, priority=-1 if args.root_load_high_priority else 0),
                "streams": [torch.cuda.Stream(dev) for _ in range(nst)],
                "side_ev": [torch.cuda.Event() for _ in range(nst)],
                "ev": torch.cuda.Event(), "ring": [torch.cuda.Event() for _ in range(max(2, F))]}
        if args.root_load == "dma":
            import ctypes
            hip = ctypes.CDLL("libamdhip64.so")
            hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                           ctypes.c_int, ctypes.c_void_p]
            hip.hipMemcpyAsync.restype = ctypes.c_int
            load["hip"] = hip
        if args.root_load == "proxy":
            import ctypes
            so = os.path.join(ROOT, "build", "ingress_proxy.so")
            if not os.path.exists(so):
                raise SystemExit("--root-load proxy needs %s (hipcc --offload-arch=gfx950 -O3 -shared "
                                 "-fPIC tools/ingress_proxy.hip -o %s)" % (so, so))
            load["proxy"] = ctypes.CDLL(so)
            load["proxy"].ingress_proxy_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p,
                                                           ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]

    def issue_load(k):
        # one ingress per step, every step, with the gather pipeline's back pressure (a band
        # buffer is rewritten only after the gather that read it, max(2, F) steps back, is
        # done: step() waits on ring[k % len])
        ls = load["stream"]
        with torch.cuda.stream(ls):
            if load["mode"] == "kernel":
                torch.bitwise_or(load["src"], 0, out=load["dst"])  # a CU kernel: read + write
            elif load["mode"] == "proxy":
                rc = load["proxy"].ingress_proxy_launch(load["dst"].data_ptr(), load["src"].data_ptr(),
                                                        load["bytes_per_step"], args.root_load_wgs,
                                                        ls.cuda_stream)
                if rc:
                    raise RuntimeError("ingress_proxy_launch failed: %d" % rc)
            else:
                # the copy engines (kind 1024 = hipMemcpyDeviceToDeviceNoCU: no CU blit kernel),
                # the bytes split over the side streams, joined back on the load stream
                nst = len(load["streams"])
                per = (load["bytes_per_step"] // nst + 255) // 256 * 256
                load["ev"].record(ls)
                for i, ss in enumerate(load["streams"]):
                    off = i * per
                    cnt = min(per, load["bytes_per_step"] - off)
                    if cnt <= 0:
                        continue
                    ss.wait_event(load["ev"])
                    rc = load["hip"].hipMemcpyAsync(load["dst"].data_ptr() + off,
                                                    load["src"].data_ptr() + off, cnt, 1024,
                                                    ss.cuda_stream)
                    if rc:
                        raise RuntimeError("hipMemcpyAsync (root-load dma) failed: %d" % rc)
                    load["side_ev"][i].record(ss)
                    ls.wait_event(load["side_ev"][i])
            load["ring"][k % len(load["ring"])].record(ls)
        load["issued"] += 1

    def step():
        k = state["k"]
        state["k"] += 1
        f = k % F  # frame slot: engine + stream
        with torch.cuda.stream(streams[f]):
            if not gather:
                timed_load = load is not None and state.get("timed")
                ring = load["ring"] if timed_load else None
                if timed_load and k - state["k0"] >= len(ring):
                    torch.cuda.current_stream(dev).wait_event(ring[k % len(ring)])
                engines[f].match(s0, s1, mcfg, out=outs[f], corrmap=corrs[f])
                if timed_load:
                    issue_load(k)
                return
            if dma is not None:
                dma_step(k, f)
                return
            i = k % NB
            if pending[i] is not None:
                land(i)  # this stream waits for the gather that last read sends[i]
            buf = sends[i]
            if nccl:
                engines[f].match(s0, s1, mcfg, out=disp_view(buf)[:rows],
                                 corrmap=corr_view(buf)[:rows] if has_corr else None)
            else:
                engines[f].match(s0, s1, mcfg, out=outs[f], corrmap=corrs[f])
                disp_view(buf)[:rows].copy_(outs[f])
                if has_corr:
                    corr_view(buf)[:rows].copy_(corrs[f])
            # the collective is ordered after this stream's match
            pending[i] = dist.gather(buf, recvs[i], dst=0, async_op=True)

    def drain():
        if gather:
            for k in range(state["k"] - NB, state["k"]):  # oldest gather first
                if k >= 0 and pending[k % NB] is not None:
                    land(k % NB)

    # Untimed warm-up. First a clock spin-up: at least --spinup-ms of back-to-back local
    # matches (no collectives, so ranks need not agree on a count). The GPU's clocks ramp
    # for ~25 ms under this load (rocprof trace in profiles/: the search kernel goes from
    # 1.78 to 1.56 ms over its first 13 launches), and K timed steps right after 3 warm-up
    # matches would average part of that ramp into a steady-state frame rate. Then the W
    # regular warm-up steps (with the gather), identical on every rank.
    t_warm = time.perf_counter()
    spins = 0
    while (time.perf_counter() - t_warm) * 1e3 < args.spinup_ms:
        for _ in range(4):
            eng.match(s0, s1, mcfg, out=out, corrmap=corr)
        spins += 4
        torch.cuda.synchronize(dev)
    for _ in range(args.warmup):
        step()
    drain()
    torch.cuda.synchronize(dev)
    warm_ms = (time.perf_counter() - t_warm) * 1e3
    if world > 1:
        dist.barrier()
    state["timed"] = True
    state["k0"] = state["k"]
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    drain()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if nccl else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # ---- after the timed region: the gather alone, then the gathered frames verified
    gather_info = None
    verify = None
    if not gather:
        gather_choice = None
    if gather:
        if dma is not None:
            gather_info = time_dma_exchange(dist, torch, dev, rank, world, dma, streams[0], nbytes)
            if nccl:  # the RCCL gather of the same buffers beside it (both timed)
                gather_info["rccl_gather_alone"] = time_gather(dist, torch, dev, nccl, rank,
                                                               sends[0], recvs[0], nbytes, world)
        else:
            gather_info = time_gather(dist, torch, dev, nccl, rank, sends[0], recvs[0], nbytes, world)
            if want_dma and nccl:
                gather_info["dma_exchange"] = (
                    "not chosen: %s" % json.dumps(gather_choice) if gather_choice
                    else "unavailable: the copy-engine setup failed")
        if not args.no_verify_gather:
            verify = verify_gather(args, C, dist, torch, np, dev, nccl, rank, world, eng, mcfg,
                                   step, drain, NB, recv_all, frame_disps, disp_view, corr_view,
                                   i16, has_corr)

    # pixels of one step over the whole job: the frame (strong scaling), a frame per rank
    # (weak), or the band itself (--band-of profiling)
    frames_px = rows * W if args.band_of > 1 else H * W * (world if args.scaling == "weak" else 1)
    value = frames_px * args.steps / elapsed / 1e6
    ms_per_step = elapsed / args.steps * 1e3

    # one match at a time on one stream (this rank's band, no gather): the latency of a
    # frame, reported beside the pipelined throughput
    serial = []
    for _ in range(3):
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        for _ in range(10):
            eng.match(s0, s1, mcfg, out=out, corrmap=corr)
        torch.cuda.synchronize(dev)
        serial.append((time.perf_counter() - t1) / 10 * 1e3)
    ms_serial = sorted(serial)[1]

    # (--kernel-reps 0: no back-to-back kernel loops -- the PMC passes use it, so every
    # dispatch they count is an in-frame one)
    roof = kernel_roofline(args, C, torch, dev, eng, mcfg, s0, s1, rows, W, n, words, world,
                           ms_per_step, frames_px) if args.kernel_reps > 0 else None

    # The CPU baseline runs at N = 1 only (one rank, after its GPU work is done, so every
    # host core is the baseline's); N > 1 lines carry null.
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(C, args.cpu_seconds)
    hp = None
    if rank == 0 and world == 1 and not args.no_host_path:
        hp = host_path(C, mcfg, reps=5)

    if rank == 0:
        if gather and args.gather_rehearsal:
            par = ("rehearsal: the row-band gather path on a 1-rank %s process group (self-"
                   "gather; not a measurement)" % ("RCCL" if nccl else "gloo"))
        elif gather and dma is not None:
            par = ("row-bands x%d + copy-engine gather over xGMI (hipMemcpyAsync into rank 0's "
                   "IPC-mapped slots, RCCL all_reduce per step)" % world if nccl else
                   "gloo rehearsal: row-bands x%d + copy-engine gather (IPC), ranks sharing %d "
                   "GPU(s) (not a measurement)" % (world, ndev))
        elif gather:
            par = ("row-bands x%d + RCCL gather over xGMI" % world if nccl else
                   "gloo rehearsal: row-bands x%d + gloo gather, ranks sharing %d GPU(s) "
                   "(not a measurement)" % (world, ndev))
        elif args.band_of > 1:
            par = "single GPU, band 0 of %d (%d rows; profiling)" % (args.band_of, rows)
        else:
            par = "replicas x%d" % world if world > 1 else "single GPU"
        line = {
            "metric": "disparity Mpix/s + ms/match, %dx2 stack @ %dx%d, 1/2/4/8 MI355X" % (n, W, H),
            "value": round(value, 2),
            "unit": "Mpix/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "spinup_matches": spins,
            "warmup_ms": round(warm_ms, 1),
            "ms_per_step": round(ms_per_step, 4),
            "frames_in_flight": F,
            "ms_per_match_one_at_a_time": round(ms_serial, 4),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (splitmix64 planted-disparity stereo, seed 0x600DF00D)",
            "config": {
                "workload": "%s: %s" % (args.config, C["desc"]),
                "n_images": n, "rows": H, "cols": W, "descriptor_bits": 32 * words,
                "rows_per_rank": rows,
                "parallelism": par,
                "backend": args.backend if dist_on else None,
                "match_config": C["cfg"],
            },
            "roofline": roof,
            "gather": gather_info,
            "gather_choice": gather_choice,
            "root_load": None if load is None else {
                "mode": load["mode"], "bytes_per_step": load["bytes_per_step"],
                "loads_issued": load["issued"], "steps_skipped": load["skipped"],
                "ingress_GBps": round(load["bytes_per_step"] * load["issued"] / elapsed / 1e9, 1),
                "workgroups": args.root_load_wgs if load["mode"] == "proxy" else None,
                "copy_streams": len(load["streams"]) if load["mode"] == "dma" else None,
                "high_priority_stream": bool(args.root_load_high_priority),
                "back_pressure": True,
                "what": "rank 0's gather ingress of an N = %d run rehearsed on one GPU: the other "
                        "%d bands' packed maps written per step into a root buffer on a side "
                        "stream (%s)" % (args.band_of, args.band_of - 1,
                                         "full-grid torch copy kernel" if load["mode"] == "kernel" else
                                         "%d long-lived copy workgroups, RCCL's receive shape" %
                                         args.root_load_wgs if load["mode"] == "proxy" else
                                         "copy engines, hipMemcpyAsync hipMemcpyDeviceToDeviceNoCU "
                                         "from a second HBM buffer on %d streams (reads and writes "
                                         "rank 0's HBM: twice the real ingress's HBM bytes)"
                                         % len(load["streams"]))},
            "verify_gather": verify,
            "cpu_baseline": cpu,
            "host_path": hp,
        }
        if "published" in C:
            pub = C["published"]
            # the published figures are one match at a time, so the speedup is
            # taken against our one-at-a-time latency; the pipelined throughput is beside it
            line["vs_published"] = dict(
                pub, ours_ms_one_at_a_time=round(ms_serial, 4),
                speedup=round(pub["ms_per_match"] / ms_serial, 1),
                ours_ms_per_step_pipelined=round(ms_per_step, 4),
                throughput_speedup=round(pub["ms_per_match"] / ms_per_step, 1))
        print(json.dumps(line), flush=True)
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()


def setup_dma_gather(args, dist, torch, dev, nccl, rank, world, recv_all, sends, nbytes):
    """The copy-engine gather (--gather dma|auto). Rank 0 shares its receive slots
    (recv_all[i], [world, nbytes] bytes on its GPU) through CUDA/HIP IPC (torch's own tensor
    sharing: the handles go out with broadcast_object_list); every other rank maps them and,
    per step, copies its packed band into its row of the slot with ONE hipMemcpyAsync on its
    own stream -- the sending GPU's copy engines over xGMI, nothing on rank 0's CUs (an RCCL
    gather receives on them: profiles/root_gather_r05.jsonl) -- then joins a one-element
    all_reduce on that stream (RCCL: stream-ordered behind the copy on every rank, so its
    completion on rank 0 means every band has landed). Slot reuse (bench.main dma_step): step
    k first waits for the all_reduce of step k-2 (rank 0 then lands frame k-2); with NB >= 4
    slots, slot k % NB last held frame k-NB, landed at step k-NB+2 <= k-2 before rank 0's
    all_reduce of that step, which step k has waited for.

    A self-test (each rank writes a pattern into its row of slot 0, rank 0 checks every row)
    runs first; any failure on any rank returns None on every rank and the RCCL gather is used
    (--gather auto), or exits (--gather dma). Returns {"copy", "signal", "remote"}."""
    import ctypes
    ok = True
    why = ""
    remote = None
    copy_fn = None
    try:
        from torch.multiprocessing.reductions import rebuild_cuda_tensor, reduce_tensor
        objs = [reduce_tensor(r)[1] if rank == 0 else None for r in recv_all]
    except Exception as ex:  # noqa: BLE001 -- any failure falls back to the RCCL gather
        ok, why, objs = False, "share: %s" % ex, [None] * len(recv_all)
    flag = torch.tensor([1.0 if ok else 0.0], device=dev if nccl else "cpu")
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if flag.item() == 1.0:
        dist.broadcast_object_list(objs, src=0)
        try:
            if rank != 0:
                remote = [rebuild_cuda_tensor(*o) for o in objs]
            hip = ctypes.CDLL("libamdhip64.so")
            hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                           ctypes.c_int, ctypes.c_void_p]
            hip.hipMemcpyAsync.restype = ctypes.c_int

            def copy_fn(i, stream):
                # kind 1024 = hipMemcpyDeviceToDeviceNoCU: the copy engines, never a blit kernel
                # on either GPU's compute units
                rc = hip.hipMemcpyAsync(remote[i][rank].data_ptr(), sends[i].data_ptr(), nbytes,
                                        1024, stream.cuda_stream)
                if rc != 0:
                    raise RuntimeError("hipMemcpyAsync (dma gather) failed: %d" % rc)
            # self-test: a rank-specific pattern through slot 0
            torch.cuda.synchronize(dev)
            if rank != 0:
                sends[0].fill_(rank * 37 % 251 + 1)
                st = torch.cuda.current_stream(dev)
                copy_fn(0, st)
                st.synchronize()
        except Exception as ex:  # noqa: BLE001
            ok, why = False, "map / copy: %s" % ex
    else:
        ok = False
    flag = torch.tensor([1.0 if ok else 0.0], device=dev if nccl else "cpu")
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    ok = flag.item() == 1.0
    if ok and rank == 0:
        torch.cuda.synchronize(dev)
        for r in range(1, world):
            if not bool((recv_all[0][r] == (r * 37 % 251 + 1)).all().item()):
                ok, why = False, "self-test: rank %d's row did not land" % r
                break
    flag = torch.tensor([1.0 if ok else 0.0], device=dev if nccl else "cpu")
    dist.broadcast(flag, src=0)
    ok = ok and flag.item() == 1.0 if rank == 0 else flag.item() == 1.0
    if not ok:
        if args.gather == "dma":
            raise SystemExit("--gather dma: setup failed (%s)" % (why or "on another rank"))
        if rank == 0:
            print("gather: copy-engine setup failed (%s); using the RCCL gather" %
                  (why or "on another rank"), file=sys.stderr)
        return None
    sigs = [torch.zeros(1, device=dev if nccl else "cpu") for _ in range(len(recv_all))]

    def signal(i, stream):
        if nccl:  # stream-ordered behind the copy (we are inside torch.cuda.stream(stream))
            return dist.all_reduce(sigs[i], async_op=True)
        stream.synchronize()  # gloo (rehearsal): the copy is done before the host joins
        return dist.all_reduce(sigs[i], async_op=True)
    return {"copy": copy_fn, "signal": signal, "remote": remote}


def time_dma_exchange(dist, torch, dev, rank, world, dma, stream, nbytes, reps=10):
    """The copy-engine exchange alone (untimed region): per rep, a barrier, then every rank
    but 0 copies one band into rank 0's slot 0 and all ranks join the signalling all_reduce;
    host wall time until it completes on this rank, median, max over ranks."""
    ts = []
    for _ in range(reps):
        dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        with torch.cuda.stream(stream):
            if rank != 0:
                dma["copy"](0, stream)
            w = dma["signal"](0, stream)
        w.wait()
        torch.cuda.synchronize(dev)
        ts.append(time.perf_counter() - t0)
    t = sorted(ts)[len(ts) // 2]
    tt = torch.tensor([t], dtype=torch.float64, device=dev if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    t = float(tt.item())
    return {"mode": "dma", "ms_per_exchange": round(t * 1e3, 4), "bytes_per_rank": nbytes,
            "bytes_to_root": nbytes * (world - 1),
            "GBps_into_root": round(nbytes * (world - 1) / t / 1e9, 1),
            "what": "every rank but 0 copies its packed band into rank 0's IPC-mapped slot "
                    "(hipMemcpyAsync on its own stream) + one-element all_reduce, host wall time "
                    "incl. launch, median of %d, max over ranks" % reps}


def time_gather(dist, torch, dev, nccl, rank, send, recv, nbytes, world, reps=10):
    """The per-step gather alone (untimed region): median of `reps` synchronous gathers of one
    packed band buffer to rank 0, each after a barrier. RCCL: HIP events on the current
    stream around the collective (the RCCL stream waits for the first, the second waits for
    the RCCL stream); gloo: host wall time."""
    ts = []
    for _ in range(reps):
        dist.barrier()
        if nccl:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            dist.gather(send, recv, dst=0)
            e1.record()
            torch.cuda.synchronize(dev)
            ts.append(e0.elapsed_time(e1))
        else:
            t = time.perf_counter()
            dist.gather(send, recv, dst=0)
            ts.append((time.perf_counter() - t) * 1e3)
    ms = sorted(ts)[len(ts) // 2]
    to_root = (world - 1) * nbytes
    return {"ms": round(ms, 4), "bytes_per_rank": nbytes, "bytes_to_root": to_root,
            "GBps_into_root": round(to_root / (ms * 1e-3) / 1e9, 1),
            "what": "median of %d synchronous gathers of the packed [disparity | corrmap] band "
                    "buffer (%s), measured on rank %d after the timed region; inside the timed "
                    "region the gather of step k overlaps the kernels of step k+1" %
                    (reps, "RCCL, HIP events on the current stream" if nccl else "gloo, host "
                     "wall time", rank)}


def _frame_fixture(name):
    """The oracle's whole-frame hashes for a BASELINE config (tests/golden/frames.json, data
    written by tests/golden/make_frames.py), or None."""
    path = os.path.join(ROOT, "tests", "golden", "frames.json")
    try:
        return json.load(open(path)).get(name)
    except (OSError, ValueError):
        return None


def verify_gather(args, C, dist, torch, np, dev, nccl, rank, world, eng, mcfg, step, drain, NB,
                  recv_all, frame_disps, disp_view, corr_view, i16, has_corr):
    """Untimed: every gather slot's receive buffer (and rank 0's float frame) is overwritten
    with a sentinel, NB more steps run with the same pipeline as the timed ones, and rank 0
    checks every slot's gathered frame: against the oracle's whole-frame sha256 for the
    config (tests/golden/frames.json) when it has one, else byte for byte against a one-GPU
    match of the whole frame. A slot that did not land, landed stale or out of order keeps
    the sentinel and fails. All ranks learn the verdict; a failure exits non-zero."""
    import hashlib
    from libbicos_amd.distributed import band_rows
    from libbicos_amd.synthetic import stereo_stack
    n, H, W = C["n"], C["H"], C["W"]
    torch.cuda.synchronize(dev)
    if rank == 0:
        for i in range(NB):
            recv_all[i].fill_(0xFF)
            if frame_disps is not None:
                frame_disps[i].fill_(float("nan"))
    dist.barrier()
    for _ in range(NB):
        step()
    drain()
    torch.cuda.synchronize(dev)
    ok, how = True, None
    if rank == 0:
        fx = _frame_fixture(args.config)
        ref = None
        if fx is None or (fx["n"], fx["H"], fx["W"]) != (n, H, W):
            FL, FR = stereo_stack(n, H, W, np.uint8, row_begin=0, row_end=H)
            fd, fc = eng.match(torch.from_numpy(FL).to(dev), torch.from_numpy(FR).to(dev), mcfg)
            ref = (fd.cpu().numpy(), None if fc is None else fc.cpu().numpy())
            how = "byte-identical to a one-GPU match of the whole frame"
        else:
            how = "sha256 of the whole frame == the oracle's (tests/golden/frames.json)"
        for i in range(NB):
            dmap = (frame_disps[i] if i16 else disp_view(recv_all[i])).cpu().numpy()
            cmap = corr_view(recv_all[i]).cpu().numpy() if has_corr else None
            parts_d, parts_c = [], []
            for r in range(world):
                rb, re_ = band_rows(H, world, r)
                parts_d.append(dmap[r, :re_ - rb])
                if has_corr:
                    parts_c.append(cmap[r, :re_ - rb])
            fd_ = np.ascontiguousarray(np.concatenate(parts_d))
            fc_ = np.ascontiguousarray(np.concatenate(parts_c)) if has_corr else None
            if ref is None:
                sha = lambda a: hashlib.sha256(a.tobytes()).hexdigest()  # noqa: E731
                good = sha(fd_) == fx["disparity_sha256"] and (
                    not has_corr or sha(fc_) == fx["corrmap_sha256"])
            else:
                good = fd_.tobytes() == ref[0].tobytes() and (
                    not has_corr or fc_.tobytes() == ref[1].tobytes())
            if not good:
                ok = False
                how = "slot %d of %d: gathered frame differs (%s)" % (i, NB, how)
                break
    flag = torch.tensor([1.0 if ok else 0.0], device=dev if nccl else "cpu")
    dist.broadcast(flag, src=0)
    if flag.item() != 1.0:
        raise SystemExit("verify-gather failed: %s" % (how or "see rank 0"))
    if rank == 0:
        print("verify-gather: %d slots x %d bands, %s" % (NB, world, how), file=sys.stderr)
    return {"ok": True, "slots": NB, "bands": world, "check": how}


def kernel_roofline(args, C, torch, dev, eng, mcfg, s0, s1, rows, W, n, words, world,
                    ms_per_step, step_px):
    """The dominant launch of the match and the HBM-bound stages, timed with HIP events on
    the stream they run on, against their rooflines; PMC HBM bytes from
    profiles/ when they were measured on these sources; the whole match's HBM-read fraction.

    In the frame: per rep both transforms, then EXACTLY the launches
    the match issues after its transform (bicos_search_agree_device: for cfg1 / cfg2 / cfg5
    one fused search + agree launch, bicos_match_plan PLAN_AGREE_IN_SEARCH), with events
    around them. Where that is one fused launch it is the line's kernel; elsewhere the search
    alone, timed the same way, is (the stage time beside it)."""
    from libbicos_amd import _lib, device
    st = torch.cuda.current_stream(dev)
    d0 = eng.transform(s0, mcfg.mode, words)
    d1 = eng.transform(s1, mcfg.mode, words)
    raw = torch.empty((rows, W), dtype=torch.int16, device=dev)
    flags = (2 | (1 if mcfg.no_dupes else 0)) if mcfg.variant == 1 else 1
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
    mc = C["cfg"]
    mv = mc.get("min_variance")
    mv = None if mv is None or mv < 0 else mv * n
    ubits = device.used_bits(n, mcfg.mode)
    sbits = transform_bits(n, mcfg.mode)
    plan = eng.plan(s0, s1, mcfg)
    fused = bool(plan & _lib.PLAN_AGREE_IN_SEARCH)
    thr = mc.get("nxcorr_threshold")
    has_corr = thr is not None
    st_out = torch.empty((rows, W), dtype=torch.float32 if has_corr else torch.int16, device=dev)
    st_corr = torch.empty((rows, W), dtype=torch.float64 if mcfg.precision else torch.float32,
                          device=dev) if has_corr else None

    one_pass = bool(plan & getattr(_lib, "PLAN_CONSISTENCY_ONE_PASS", 0))

    def search_launch():
        # with the set-bits hint the pipeline passes (engine.cpp match_device)
        eng.search(d0, d1, W, words, flags, mcfg.max_lr_diff, out=raw, bits=sbits)

    def stage_launch():  # the match past its transform (bicos_search_agree_device)
        eng.search_agree(d0, d1, s0, s1, mcfg, out=st_out, corrmap=st_corr)

    reps = args.kernel_reps
    search_launch()  # warm
    stage_launch()
    # in the frame: the search alone (its own events), then the post-transform stage
    fe = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for a, b in fe:
        eng.transform(s0, mcfg.mode, words, out=d0)
        eng.transform(s1, mcfg.mode, words, out=d1)
        a.record(st)
        search_launch()
        b.record(st)
        if thr is not None:
            eng.agree(raw, s0, s1, thr, minvar_scaled=mv, step=mc.get("subpixel_step"))
    fs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for a, b in fs:
        eng.transform(s0, mcfg.mode, words, out=d0)
        eng.transform(s1, mcfg.mode, words, out=d1)
        a.record(st)
        stage_launch()
        b.record(st)
    ev[0].record(st)
    for _ in range(reps):
        search_launch()
    ev[1].record(st)
    for _ in range(reps):
        eng.transform(s0, mcfg.mode, words, out=d0)
    ev[2].record(st)
    stage = "subpixel" if mc.get("subpixel_step") else "nxcorr"
    ev[3].record(st)
    for _ in range(reps):
        eng.agree(raw, s0, s1, 0.96 if thr is None else thr, minvar_scaled=mv,
                  step=mc.get("subpixel_step"))
    ev[4].record(st)
    torch.cuda.synchronize(dev)
    t_b2b = ev[0].elapsed_time(ev[1]) / reps * 1e-3
    in_frame = [a.elapsed_time(b) * 1e-3 for a, b in fe]
    t_search = sum(in_frame) / len(in_frame)  # the in-frame average
    st_frame = [a.elapsed_time(b) * 1e-3 for a, b in fs]
    t_stage = sum(st_frame) / len(st_frame)
    t_tf = ev[1].elapsed_time(ev[2]) / reps * 1e-3
    t_agree = ev[3].elapsed_time(ev[4]) / reps * 1e-3
    pairs = search_pairs(rows, W, mc)
    # HBM stages, algorithmic bytes: transform reads n B/px and writes 4w B/px (one stack);
    # agree reads the int16 raw disparity + 2n B per valid px, writes 8 B/px (disp + corr)
    tf_bytes = rows * W * (n + 4 * words)
    valid = float((raw != -32768).float().mean().item())
    ag_bytes = rows * W * (2 + 8) + rows * W * valid * 2 * n
    # algorithmic bytes of the search stage: both descriptor bands + the int16 output per pass
    # (Consistency: forward + reverse pass, then the check reads both index maps and writes
    # the disparity, 6 B per pixel)
    search_bytes = rows * W * (2 * 4 * words + 2) * (2 if mc.get("variant", 0) == 1 else 1) + \
        (rows * W * 6 if mc.get("variant", 0) == 1 else 0)
    if one_pass:  # one launch: both descriptor bands in, the checked disparity out
        search_bytes = rows * W * (2 * 4 * words + 2)
    mx = mx_search()
    cons = mc.get("variant", 0) == 1
    nodupes = not cons or bool(mc.get("no_dupes", False))
    pk = bool(plan & _lib.PLAN_PACKED_KEYS)
    kname = ("search_pk_kernel" if pk else "search_mx_kernel") if mx else "search16_kernel"
    if one_pass:
        kname = "search_lr_kernel"
    cfgname = args.config
    # the search stage's bytes per frame: every search dispatch (tail launches, both
    # Consistency passes, the reverse list) and Consistency's check kernel
    traffic = load_traffic((kname, "consistency_kernel") if cons and not one_pass else kname,
                           cfgname, rows)
    # Consistency: the distinct col1 the forward search keeps, over which the reverse search
    # runs (engine.cpp reverse_search)
    kept = None
    if one_pass:
        kept = 0.0  # the reverse search reuses the forward products: no pairs of its own
    elif cons and mx:
        fwd = torch.empty_like(raw)
        eng.search(d0, d1, W, words, 1 if nodupes else 0, -1, out=fwd, bits=ubits)
        c0 = torch.arange(W, device=dev, dtype=torch.int64).expand(rows, W)
        ok = fwd != -32768
        mark = torch.zeros((rows, W + 1), dtype=torch.bool, device=dev)
        mark.scatter_(1, torch.where(ok, c0 - fwd.long(), torch.full_like(c0, W)), True)
        kept = float(mark[:, :W].sum().item())
        if plan & _lib.PLAN_DENSE_ROWS:
            # dense-row fast path: rows whose forward search kept >= 7/8 of their col0 search
            # every col0 in the reverse pass (search_mx.hip dense_row)
            dense = ok.sum(dim=1) * 8 >= 7 * W
            kept = float(torch.where(dense, torch.full_like(mark[:, 0], W, dtype=torch.int64),
                                     mark[:, :W].sum(dim=1)).sum().item())
    if mx:
        alg_flops, used_flops = mx_flops(rows, W, words, mc, ubits, sbits, reverse_col1=kept)
        kpeak = (lr_key_pair_peak(2 if os.environ.get("BICOS_LR_T") == "2" else 4) if one_pass else
                 pk_key_pair_peak() if pk else
                 mx_key_pair_peak(words, mc, mx_reach_planted(W))) / 1e9
        evaluated = pairs + (kept if kept is not None else pairs / W) * W if cons else pairs
        k_exec = int(round(alg_flops / (2 * evaluated)))
        # the launch the line is about: the fused search + agree (the match's own launch) or
        # the search alone
        t_main = t_stage if fused else t_search
        t_fp4 = alg_flops / (MFMA_FP4_DENSE_TFLOPS * 1e12)      # the matrix-core floor
        t_key = evaluated / (kpeak * 1e9)                       # the key reduction as executed
        t_ag = ag_bytes / (HBM_PEAK_GBS * 1e9) if fused else 0.0  # the fused agree's bytes
        bound = "valu" if t_key > t_fp4 else "mfma"
        t_bound = max(t_fp4, t_key) + t_ag
        achieved_tf = alg_flops / t_main / 1e12
        fp4 = {"achieved": round(achieved_tf, 1), "peak": MFMA_FP4_DENSE_TFLOPS, "unit": "TFLOP/s",
               "frac": round(achieved_tf / MFMA_FP4_DENSE_TFLOPS, 4)}
        kview = {"achieved": round(evaluated / t_main / 1e9, 1), "peak": round(kpeak, 1),
                 "unit": "Gpairs/s", "frac": round(t_key / t_main, 4)}
        if one_pass:
            kname_long = ("search_lr_kernel<%d words> (Consistency in one launch: the forward and "
                          "the reverse FP4 MFMA Hamming argmin from one set of products, the "
                          "left-right check in the same workgroup)" % words)
        elif fused:
            kname_long = ("search_pk_kernel<1 word, AG> (packed-key FP4 MFMA search with the NXC "
                          "agree of its col0 in the same launch)" if pk else
                          "search_mx_kernel<%d words, AG> (FP4 MFMA Hamming argmin with the NXC "
                          "agree of its col0 in the same launch)" % words)
        else:
            kname_long = (("search_pk_kernel<%d words> x2 (forward + reverse over the kept col1)"
                           if pk else
                           "search_mx_kernel<%d words> x2 (forward + reverse FP4 MFMA Hamming argmin "
                           "over the kept col1)") % words
                          if cons else
                          "search_pk_kernel<%d words> (FP4 MFMA Hamming products, two distances per "
                          "accumulator register, v_pk_minimum3_f16 trees)" % words if pk else
                          "search_mx_kernel<%d words> (FP4 MFMA Hamming products, argmin keys in the "
                          "accumulator)" % words)
        # frac = the launch's bound time over its measured time: max(matrix-core floor, key
        # reduction issue as executed) + the fused agree's bytes at 8 TB/s. achieved / peak in
        # pairs/s so that achieved / peak = frac: peak = the pairs the bound would evaluate in
        # the launch time.
        roof = {
            "kernel": kname_long,
            "bound": bound,
            "achieved": round(evaluated / t_main / 1e9, 1),
            "peak": round(evaluated / t_bound / 1e9, 1),
            "unit": "Gpairs/s",
            "frac": round(t_bound / t_main, 4),
            "bound_model": {
                "what": "max(FP4 floor, VALU key reduction as executed)%s over the launch time"
                        % (" + the fused agree's algorithmic bytes at 8 TB/s" if fused else ""),
                "fp4_floor_ms": round(t_fp4 * 1e3, 4),
                "key_reduction_ms": round(t_key * 1e3, 4),
                "agree_hbm_ms": round(t_ag * 1e3, 4),
                "bound_ms": round(t_bound * 1e3, 4),
                "key_model": ("lr_key_pair_peak: 96 half-rate + 26 full-rate instructions per wave "
                              "and block of 4 tiles (both directions' reductions)" if one_pass else
                              "pk_key_pair_peak: 10 half-rate + 1 full-rate lane-ops per lane, wide "
                              "tile and block" if pk else
                              "mx_key_pair_peak: the ISA's VALU per (wave, tile, block), the "
                              "last-minimum tree weighted by the planted frame's reach fraction "
                              "%.3f (tools/reach_sim.py); DESIGN.md s5.1" % mx_reach_planted(W)),
            },
            "timing": ("in frame: the average of %d launches timed with HIP events on their stream, "
                       "each after both transforms, exactly as the match issues them "
                       "(bicos_search_agree_device)" % reps) if fused else
                      ("in frame: the average of %d searches timed with HIP events on their "
                       "stream, each after both transforms and before the agree, as in a match"
                       % reps),
            "ms_per_launch": round(t_main * 1e3, 4),
            "agree_fused_in_match": fused,
            "plan": plan,
            "stage_after_transform_ms": round(t_stage * 1e3, 4),
            "search_alone_in_frame": {
                "ms": round(t_search * 1e3, 4),
                "fp4_frac": round(alg_flops / t_search / 1e12 / MFMA_FP4_DENSE_TFLOPS, 4),
                "back_to_back_ms": round(t_b2b * 1e3, 4),
                "what": "the search launch alone (bicos_search_device), a secondary view" if fused
                        else "= this line's kernel",
            },
            "fp4_only_view": dict(fp4, what="the launch time against the dense FP4 MFMA peak alone "
                                            "(2 x K FLOPs per pair)"),
            "fp4_combined_view": {
                "frac": round((t_fp4 + t_ag) / t_main, 4),
                "what": "FP4 floor%s over the launch time" % (" + agree bytes at 8 TB/s" if fused else ""),
            },
            "key_reduction_view": dict(kview, what="the VALU key reduction as executed (issue bound "
                                                   "at the measured rates), alone"),
            # gfx950 runs the MFMAs and the VALU of the waves sharing a SIMD one after the other
            # (profiles/mfma_valu_overlap_r06.jsonl: an MFMA wave + a VALU wave on one SIMD take
            # the SUM of their times, FP4 and bf16 alike), so the launch's floor is the sum
            "serial_view": {
                "ms": round((t_fp4 + t_key + t_ag) * 1e3, 4),
                "frac": round((t_fp4 + t_key + t_ag) / t_main, 4),
                "what": "FP4 floor + key reduction as executed%s, added: the matrix pipe and the "
                        "VALU of one SIMD serialize (tools/mfma_valu_overlap.hip, "
                        "profiles/mfma_valu_overlap_r06.jsonl)" % (" + agree bytes" if fused else ""),
            },
            "all_trees_view": None if pk else {
                "peak": round(mx_key_pair_peak_all_trees() / 1e9, 1),
                "frac": round(evaluated / mx_key_pair_peak_all_trees() / t_main, 4),
                "what": "round 5's key-reduction model (both trees on every pair): an upper bound "
                        "of the VALU work, 2.1x the executed count at cfg2 (DESIGN.md s5.1)",
            },
            "reverse_col1_kept": kept,
            "traffic": traffic["bytes"],
            "traffic_source": traffic.get("source") or traffic.get("why"),
            # fused: the PMC bytes are the one launch's, search + agree, against both stages'
            # algorithmic bytes
            "traffic_covers": "search + agree (one fused launch)" if fused else "search",
            "algorithmic_bytes_traffic_covers": search_bytes + ag_bytes if fused else search_bytes,
            "algorithmic_bytes": search_bytes + (ag_bytes if fused else 0),
            "algorithmic_flops": alg_flops,
            "k_bits_per_pair": k_exec,
            "used_bits_view": {
                "what": "the same launch time against 2 x the bits the transform sets per "
                        "descriptor (%d of %d)" % (sbits, k_exec),
                "flops": used_flops,
                "frac": round(used_flops / t_main / 1e12 / MFMA_FP4_DENSE_TFLOPS, 4),
            },
            "pairs_per_launch": evaluated,
            "peak_model": "dense FP4 MFMA peak (MI355X_MICROARCH.md); algorithmic FLOPs = 2 x K "
                          "per Hamming pair, K = the descriptor bits multiplied (the descriptor "
                          "width, less whole 64-bit K-steps above the set bits): never more "
                          "than executed",
            "sustained_view": {
                "peak": MFMA_FP4_SUSTAINED_TFLOPS,
                "frac": round(achieved_tf / MFMA_FP4_SUSTAINED_TFLOPS, 4),
                "source": "profiles/mfma_rates_r01.jsonl (tools/mfma_rate.hip, 4 waves/SIMD)",
            },
        }
    else:
        pairs *= 2 if cons else 1  # two passes with Consistency
        achieved = pairs / t_search / 1e9
        peak = search_pair_peak(words, mc) / 1e9
        roof = {
            "kernel": ("search16_kernel<%d words> x2 (forward + reverse Hamming argmin)" % words
                       if cons else
                       "search16_kernel<%d words> (Hamming argmin, packed 16-bit keys)" % words),
            "bound": "valu",
            "achieved": round(achieved, 1),
            "peak": round(peak, 1),
            "unit": "Gpairs/s",
            "frac": round(achieved / peak, 4),
            "traffic": traffic["bytes"],
            "traffic_source": traffic.get("source") or traffic.get("why"),
            "algorithmic_bytes": search_bytes,
            "pairs_per_launch": pairs,
            "ms_per_launch": round(t_search * 1e3, 4),
            "peak_model": "issue bound of the per-pair VALU mix at measured rates "
                          "(full %.1f / half %.1f T lane-op/s); see DESIGN.md s5" %
                          (VALU_FULL_TOPS, VALU_HALF_TOPS),
            "lane_ops_view": {
                "achieved_Tops": round(search_ops(rows, W, words, mc) * (2 if cons else 1) / t_search / 1e12, 2),
                "nominal_peak_Tops": round(VALU_NOMINAL_TOPS, 1),
                "ops_model": "one pass over the cost matrix, 32-bit keys: 2w+3 (2w+2) lane-ops per pair",
            },
        }
    if stage == "subpixel":
        # the refine is fp32-VALU work: per valid pixel and x step, n x (quadratic 5 +
        # round/wrap 3 + mean sum 1 + centre 1 + two fma) = 12n lane-ops, plus the step's NXC
        # (correctly rounded sqrt + division + argmax, ~30)
        xs = subpixel_steps(mc["subpixel_step"])
        sp_ops = rows * W * valid * xs * (12 * n + 30)
        ach = sp_ops / t_agree / 1e12
        roof["subpixel"] = {
            "bound": "valu (fp32)",
            "x_steps": xs,
            "lane_ops": sp_ops,
            "ops_model": "per valid px and x step: 12 x n (interp 5, round/wrap 3, sum 1, "
                         "centre 1, fma 2) + 30 (NXC sqrt/div/argmax)",
            "achieved_Tops": round(ach, 2),
            "peak_Tops": round(VALU_NOMINAL_TOPS, 1),
            "frac": round(ach / VALU_NOMINAL_TOPS, 4),
            "peak_source": "spec: 256 CUs x 128 fp32 lanes/clk x 2.4 GHz = 78.6 T lane-op/s "
                           "(MI355X_MICROARCH.md 157.3 TF fp32 / 2)",
            "measured_view": {"peak_Tops": VALU_FULL_TOPS,
                              "frac": round(ach / VALU_FULL_TOPS, 4),
                              "source": "profiles/valu_rates_r01.jsonl (full-rate ops at the "
                                        "held clock, measured)"},
            "ms": round(t_agree * 1e3, 4),
        }
    tf_tr = load_traffic("transform", cfgname, rows)
    ag_tr = load_traffic("subpixel" if stage == "subpixel" else "agree", cfgname, rows)
    roof["hbm"] = {
        "transform_GBps": round(tf_bytes / t_tf / 1e9, 1),
        "transform_frac": round(tf_bytes / t_tf / 1e9 / HBM_PEAK_GBS, 4),
        "transform_ms": round(t_tf * 1e3, 4),
        "transform_traffic": tf_tr["bytes"] and tf_tr["bytes"] / 2,  # PMC: both stacks / 2
        "agree_GBps": round(ag_bytes / t_agree / 1e9, 1),
        "agree_frac": round(ag_bytes / t_agree / 1e9 / HBM_PEAK_GBS, 4),
        "agree_ms": round(t_agree * 1e3, 4),
        "agree_traffic": ag_tr["bytes"],
        "agree_stage": stage,
        "traffic_source": tf_tr.get("source") or tf_tr.get("why"),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
    }
    # the whole match against the HBM-read roofline (the north star's unit): the bytes each
    # stage must read from HBM per frame -- both stacks (transform), both descriptor sets
    # (search), raw disparity + the samples of valid pixels (agree) -- over the whole job's
    # time per frame, against N x 8 TB/s
    P = step_px
    read_bytes = 2 * n * P + 2 * 4 * words * P + 2 * P + valid * 2 * n * P
    roof["match_hbm_read"] = {
        "bytes_per_frame": int(read_bytes),
        "achieved_GBps": round(read_bytes / (ms_per_step * 1e-3) / 1e9, 1),
        "peak_GBps": HBM_PEAK_GBS * world,
        "frac": round(read_bytes / (ms_per_step * 1e-3) / 1e9 / (HBM_PEAK_GBS * world), 4),
        "model": "transform 2nP + search 2*4wP + agree (2P + valid*2nP) bytes read per frame, "
                 "P = %d px, over ms_per_step, vs %d x 8 TB/s" % (P, world),
    }
    return roof


def host_path(C, mcfg, reps):
    """The same match from host numpy stacks to host maps (bicos_match_host: what
    BICOS_Match / pybicos.match run), PCIe transfers included. Reported beside the metric,
    never as `value` (SURVEY.md s8 d: end-to-end incl. H2D/D2H separately)."""
    import ctypes
    import numpy as np
    from libbicos_amd import _lib
    from libbicos_amd.synthetic import stereo_stack

    n, H, W = C["n"], C["H"], C["W"]
    L, R = stereo_stack(n, H, W, np.uint8)
    left = [L[t].copy() for t in range(n)]  # separately allocated images, like cv2 reads
    right = [R[t].copy() for t in range(n)]
    p0 = (ctypes.c_void_p * n)(*[a.ctypes.data for a in left])
    p1 = (ctypes.c_void_p * n)(*[a.ctypes.data for a in right])
    cfgc, has = mcfg.to_c()
    disp = np.empty((H, W), np.float32 if has else np.int16)
    corr = np.empty((H, W), np.float64 if mcfg.precision else np.float32)
    lib = _lib.lib()

    def once():
        t0 = time.perf_counter()
        _lib.check(lib.bicos_match_host(None, p0, p1, n, H, W, 0, 1, ctypes.byref(cfgc), has,
                                        disp.ctypes.data, corr.ctypes.data if has else None),
                   "bicos_match_host")
        return time.perf_counter() - t0

    once()
    ts = [once() for _ in range(reps)]
    t = float(sorted(ts)[len(ts) // 2])
    return {
        "ms_per_match": round(t * 1e3, 3),
        "value": round(H * W / t / 1e6, 1),
        "unit": "Mpix/s",
        "h2d_bytes": int(L.nbytes + R.nbytes),
        "d2h_bytes": int(disp.nbytes + (corr.nbytes if has else 0)),
        "what": "host numpy stacks (separate images) -> host maps via bicos_match_host "
                "(banded pinned upload overlapped with the match), median of %d" % reps,
    }


def host_cpu_info():
    """CPU model, logical CPUs of the machine (nproc), CPUs this process may run on
    (affinity) and the cgroup CPU quota in cores (None when unlimited)."""
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    return {"model": model, "nproc": os.cpu_count(), "affinity": affinity, "cgroup_quota": quota}


def cpu_baseline(C, seconds):
    """The C oracle (a restatement of the reference CPU path, oracle/bicos_oracle.c) on every
    host core this process may use, over a bounded row sample of the same frame: the x86-64-v3
    build (popcnt/AVX2) is `value`; the as-shipped-flags build (-O3, no -march: libgcc
    popcount, like the reference's CMake build) is timed on the same sample beside it. Rows
    are independent (SURVEY.md s8 e), so the per-frame rate is the sample's rows/s x cols."""
    import numpy as np
    from libbicos_amd.synthetic import stereo_stack
    from oracle import oracle

    n, H, W = C["n"], C["H"], C["W"]
    info = host_cpu_info()
    cores = info["affinity"]
    if info["cgroup_quota"]:
        cores = max(1, min(cores, int(info["cgroup_quota"])))
    ocfg = oracle.OracleConfig(**C["cfg"])
    probe = max(cores, 8)
    L, R = stereo_stack(n, H, W, np.uint8, row_begin=0, row_end=probe)
    t = time.perf_counter()
    oracle.match(L, R, ocfg, nthreads=cores, variant="v3")
    per_row = (time.perf_counter() - t) / probe
    # `seconds` of CPU time per build (wall = seconds / cores): a row sample of the frame, or
    # whole frames repeated when one frame takes less than that
    wall = seconds / cores
    rows = int(max(probe, min(H, wall / max(per_row, 1e-9))))
    rows = min(H, max(cores, rows // cores * cores))
    L, R = stereo_stack(n, H, W, np.uint8, row_begin=0, row_end=rows)

    def timed(variant, budget):
        reps, el = 0, 0.0
        while reps == 0 or el < budget:
            t = time.perf_counter()
            oracle.match(L, R, ocfg, nthreads=cores, variant=variant)
            el += time.perf_counter() - t
            reps += 1
        return reps, el

    reps, el = timed("v3", wall)
    reps_s, el_s = timed("", wall)
    shipped = reps_s * rows * W / el_s / 1e6
    return {
        "value": round(reps * rows * W / el / 1e6, 4),
        "unit": "Mpix/s",
        "cores": cores,
        "kind": "port",
        "sample": "%d x %d of %d rows (x %d cols, n=%d), full match per row, %.1f s wall = %.0f "
                  "CPU-s; per-frame rate extrapolated from the row sample (rows are "
                  "independent); oracle -O3 -march=x86-64-v3 -ffp-contract=off, %d threads"
                  % (reps, rows, H, W, n, el, el * cores, cores),
        "extrapolated_from_rows": rows,
        "ms_per_match_extrapolated": round(el / reps / rows * H * 1e3, 1),
        "as_shipped_flags": {
            "value": round(shipped, 4),
            "ms_per_match_extrapolated": round(el_s / reps_s / rows * H * 1e3, 1),
            "build": "oracle -O3 -ffp-contract=off, no -march (libgcc popcount, as the "
                     "reference CMake build)",
            "sample": "%d x %d rows, %.1f s wall" % (reps_s, rows, el_s),
        },
        "host": info,
    }


if __name__ == "__main__":
    main()
