"""HBM traffic and counter ratios per kernel, from rocprofv3 PMC passes.

usage: python tools/pmc_traffic.py PMC_DIR OUT_JSON

PMC_DIR holds the counter_collection.csv files of tools/pmc_cfg_r04.sh (one
counter group per pass; FETCH_SIZE and WRITE_SIZE in their own passes).
Correction per MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE reports half the
bytes of a 16-B-per-lane read (both buffer_load and buffer_load...lds),
WRITE_SIZE is exact for 16-B stores and fp32 atomics, so HBM bytes =
2 * FETCH_SIZE + WRITE_SIZE (rocprofv3 reports KB).  Memory-side counters
include Infinity-Cache hits: an upper bound on DRAM bytes.

OUT_JSON["kernels"] has one entry per kernel symbol (per-dispatch means);
bench.py attaches roofline.traffic only from the entry whose name contains
every substring of the ``[kernel: a+b]`` marker in the dispatched variant.
OUT_JSON["classes"] groups them by the bench's timer-class names.
"""
import json
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmcsum import derived, load  # noqa: E402

# bench timer class -> alternatives, each a list of substrings that must all
# appear in the kernel name
CLASSES = {
    "ConvLSTM BPTT step": [["EpiConvLstmBwd"], ["k_convlstm_bwd_frames"], ["k_convlstm_bwd_pairs"],
                           ["k_convlstm_bwd_f32"]],
    "ConvLSTM forward step": [["EpiConvLstmFwd"], ["k_convlstm_fwd_frames"], ["k_convlstm_fwd_f32"]],
    "ConvLSTM weight-gradient GEMM": [["128, 128, 32", "LdIm2colTB", "EpiStore<true>"], ["GIm2colT", "EpiAtomicD"],
                                      ["GIm2colT", "EpiWgrad"]],
    "batched dx": [["EpiStoreBiasT"]],
}


def entry(cs):
    mean = {c: sum(v) / len(v) for c, v in cs.items()}
    out = {"dispatches": max(len(v) for v in cs.values())}
    if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
        f, w = mean["FETCH_SIZE"] * 1024.0, mean["WRITE_SIZE"] * 1024.0
        out.update({"fetch_size_bytes": f, "write_size_bytes": w, "hbm_bytes_per_launch": 2.0 * f + w,
                    "correction": "2*FETCH_SIZE + WRITE_SIZE (gfx950)"})
    out.update({k: round(v, 4) for k, v in derived(mean).items()})
    out["counters_per_dispatch"] = {c: v for c, v in mean.items() if c not in ("FETCH_SIZE", "WRITE_SIZE")}
    return out


def main():
    d, out = sys.argv[1], sys.argv[2]
    acc = load(d)
    kernels = {k: entry(cs) for k, cs in acc.items()
               if sum(cs.get("SQ_WAVE_CYCLES", [0])) > 0 or "FETCH_SIZE" in cs}
    classes = {}
    for cls, subs in CLASSES.items():
        names = [k for k in kernels if any(all(s in k for s in alt) for alt in subs)]
        if names:
            classes[cls] = {"kernels": names}
    json.dump({"source": d, "kernels": kernels, "classes": classes}, open(out, "w"), indent=1)
    for k, e in sorted(kernels.items(), key=lambda kv: -kv[1].get("hbm_bytes_per_launch", 0))[:12]:
        print(f"{e.get('hbm_bytes_per_launch', 0) / 1e6:10.1f} MB  mfma {e.get('mfma_util', 0):.3f}  "
              f"ldsconf {e.get('lds_conflict_rate', 0):.3f}  x{e['dispatches']}  {k[:100]}")


if __name__ == "__main__":
    main()
