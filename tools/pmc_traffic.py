"""HBM traffic per launch of the roofline kernel classes, from rocprofv3 PMC passes.

usage: python tools/pmc_traffic.py PMC_DIR OUT_JSON

PMC_DIR holds the counter_collection.csv files of tools/pmc.sh (FETCH_SIZE and
WRITE_SIZE in their own passes).  Correction per MI355X_MICROARCH.md §HBM:
on gfx950 FETCH_SIZE reports half the bytes of a 16-B-per-lane read (both
buffer_load and buffer_load...lds), WRITE_SIZE is exact for 16-B stores and
fp32 atomics, so HBM bytes = 2 * FETCH_SIZE + WRITE_SIZE (rocprofv3 reports KB).
Memory-side counters include Infinity-Cache hits: an upper bound on DRAM bytes.
bench.py reads OUT_JSON to fill roofline.traffic.
"""
import json
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmcsum import derived, load  # noqa: E402

# kernel class (bench.py names) -> alternatives, each a list of substrings that
# must all appear in the kernel name (fp32 register-staged / bf16 LDS-DMA ring)
CLASSES = {
    "ConvLSTM BPTT step": [["EpiConvLstmBwd"], ["k_convlstm_bwd_frames"], ["k_convlstm_bwd_pairs"]],
    "ConvLSTM forward step": [["EpiConvLstmFwd"], ["k_convlstm_fwd_frames"]],
    "ConvLSTM weight-gradient GEMM": [["128, 128, 32", "LdIm2colTB", "EpiStore<true>"], ["GIm2colT", "EpiAtomicD"],
                                      ["GIm2colT", "EpiWgrad"]],
}


def main():
    d, out = sys.argv[1], sys.argv[2]
    acc = load(d)
    res = {}
    for cls, subs in CLASSES.items():
        vals = {}
        for k, cs in acc.items():
            if any(all(s in k for s in alt) for alt in subs):
                for c, v in cs.items():
                    vals.setdefault(c, []).extend(v)
        if not vals.get("FETCH_SIZE") or not vals.get("WRITE_SIZE"):
            continue
        mean = {c: sum(v) / len(v) for c, v in vals.items()}
        f, w = mean["FETCH_SIZE"] * 1024.0, mean["WRITE_SIZE"] * 1024.0
        res[cls] = {"fetch_size_bytes": f, "write_size_bytes": w, "hbm_bytes_per_launch": 2.0 * f + w,
                    "dispatches": len(vals["FETCH_SIZE"]), "correction": "2*FETCH_SIZE + WRITE_SIZE (gfx950)",
                    **{k: round(v, 4) for k, v in derived(mean).items()},
                    "counters_per_dispatch": {c: v for c, v in mean.items() if c not in ("FETCH_SIZE", "WRITE_SIZE")}}
    json.dump({"source": d, "classes": res}, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
