"""Record this build's device glue-optimisation output (GPU box): tests/golden/gl_device_golden.json.

  python tests/golden/make_device_glue_golden.py [OUT.json]   (default: tests/golden/gl_device_golden.json;
                                                               on a gpurun box write under gpurun_out/ and copy back)

For every glue fixture of tests/test_glue.py: the optimum bits of one optimize_chains launch
(sha256 of the float32 outputs, the iteration / evaluation counters, the first and last loss
as float.hex), and the end of the device run_and_compare (every merge popped, sha256 of the
segmentation and of the geometry).  test_glue.py asserts them exactly.  Re-run after a
deliberate change of csrc/glue.h (and say why in the commit).
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "pt-bpe_amd"), REPO]

import test_glue as T  # noqa: E402


def main():
    T.CHECK_GLUE[0] = False  # (record the runs; the statistical bounds are the tests' business)
    out = {}
    for name in T.NAMES:
        out.setdefault(name, {})["opt"] = T.device_opt_record(name)[0]
    for name in T.NAMES + ["gl_pdb72_readme"] + T.PARETO:
        bpe = T.run_and_compare(name, device=True)
        out.setdefault(name, {})["run"] = T.device_run_record(bpe)
        bpe.close()
    path = sys.argv[1] if len(sys.argv) > 1 else T.DEV_GOLDEN
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(f"wrote {path}: {sorted(out)}")


if __name__ == "__main__":
    main()
