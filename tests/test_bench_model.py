"""The work models bench.py reports its rooflines with (CPU only): x-step counts of the
subpixel loop, K-steps and FLOPs of the matrix-core search, the issue-rate bounds."""
import numpy as np
import pytest

import bench


def _ref_steps(step):
    # the reference's loop, accumulated in float32 (agree.hpp:122)
    x, k = np.float32(-1.0), 0
    while x <= np.float32(1.0):
        k += 1
        x = np.float32(x + np.float32(step))
    return k


@pytest.mark.parametrize("step", [0.1, 0.25, 0.5, 0.05, 0.7, 2.0, 1.0 / 3.0])
def test_subpixel_steps_follow_the_float_loop(step):
    assert bench.subpixel_steps(step) == _ref_steps(step)


def test_subpixel_steps_known_values():
    assert bench.subpixel_steps(0.1) == 20   # 1.0000001 > 1 after 20 additions
    assert bench.subpixel_steps(0.5) == 5
    assert bench.subpixel_steps(2.0) == 2


@pytest.mark.parametrize("words,bits,ks", [(1, 25, 1), (2, 61, 1), (4, 125, 2), (8, 154, 3),
                                           (8, 192, 3), (8, 193, 4), (8, 0, 4), (4, 0, 2)])
def test_mx_ksteps(words, bits, ks):
    assert bench.mx_ksteps(words, bits) == ks


def test_mx_flops_cfg2_and_cfg4():
    """Algorithmic K never exceeds the executed K-steps (cfg4 was priced
    on 256 padded bits); the used-bit view prices the bits the transform sets."""
    cfg2 = bench.CONFIGS["cfg2"]
    alg, used = bench.mx_flops(1536, 2048, 4, cfg2["cfg"], 4 * 33 - 5, bench.transform_bits(33, 0))
    assert alg == 1536 * 2048 * 2048 * 2 * 128
    assert used == 1536 * 2048 * 2048 * 2 * 126
    cfg4 = bench.CONFIGS["cfg4"]
    alg, used = bench.mx_flops(1536, 2048, 8, cfg4["cfg"], 4 * 40 - 5, bench.transform_bits(40, 0))
    pairs = 2 * 1536 * 2048 * 2048  # forward + reverse
    assert alg == pairs * 2 * 192 and used == pairs * 2 * 154


def test_transform_bits_match_the_oracle(oracle):
    from libbicos_amd.synthetic import random_stack
    for n, mode in [(2, 0), (3, 0), (4, 0), (33, 0), (40, 0), (5, 1), (16, 1)]:
        d = oracle.transform(random_stack(n, 32, 64, seed=n), mode, 8)
        hi = max(32 * w + int(np.floor(np.log2(d[..., w][d[..., w] != 0].astype(np.float64)).max()))
                 for w in range(8) if (d[..., w] != 0).any())
        assert hi + 1 == bench.transform_bits(n, mode), (n, mode)


def test_configs_match_the_baseline():
    c = bench.CONFIGS
    assert (c["cfg2"]["n"], c["cfg2"]["H"], c["cfg2"]["W"]) == (33, 1536, 2048)
    assert c["cfg3"]["cfg"]["subpixel_step"] == 0.1 and c["cfg3"]["cfg"]["min_variance"] == 2.0
    assert c["cfg4"]["n"] >= 40 and c["cfg4"]["cfg"]["variant"] == 1
    assert (c["cfg5"]["H"], c["cfg5"]["W"]) == (2160, 3840)
    assert (c["cfg1"]["n"], c["cfg1"]["H"], c["cfg1"]["W"]) == (8, 480, 640)


def test_key_pair_bound_is_positive_and_ordered():
    # duplicate detection costs issue slots: the NoDuplicates bound is the lower one
    nd = bench.mx_key_pair_peak(4, {"variant": 0})
    cons = bench.mx_key_pair_peak(8, {"variant": 1, "no_dupes": False})
    assert 0 < nd < cons


def test_scale_model_prediction_rule(tmp_path):
    """tools/scale_model.py: step = max(rank 0's band x its measured slowdown,
    one band over one link); N = 1 is the measured whole-frame rate."""
    import json
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import scale_model
    recs = [dict(config="cfg2", band_of=8, root_load="none", ms_per_step=0.06),
            dict(config="cfg2", band_of=8, root_load="proxy16", ms_per_step=0.072),
            dict(config="cfg2", band_of=8, root_load="dma", ms_per_step=0.0612)]
    p = tmp_path / "rg.jsonl"
    p.write_text("\n".join(json.dumps(r) for r in recs))
    out = scale_model.predict(scale_model.load(str(p)), {"cfg2": 8000.0})
    by = {(o["gather"], o["link_GBps"]): o for o in out}
    band_bytes = 192 * 2048 * 6
    for link in scale_model.LINK_GBPS:
        t_link = band_bytes / (link * 1e9) * 1e3
        assert by[("rccl", link)]["predicted_ms_per_step"] == round(max(0.072, t_link), 4)
        assert by[("dma", link)]["predicted_ms_per_step"] == round(max(0.0612, t_link), 4)
    o = by[("rccl", 153.0)]
    assert o["predicted_Mpix_s"] == round(1536 * 2048 / (0.072e-3) / 1e6, 0)
    assert o["x_vs_N1"] == round(o["predicted_Mpix_s"] / 8000.0, 2)
