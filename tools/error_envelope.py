"""Write tests/golden/error_envelope.json from a GPU test run's error log.

    XALM_ERR_LOG=gpurun_out/err_log.json python -m pytest tests -m gpu ...   (on the GPU box)
    python tools/error_envelope.py gpurun_out/err_log.json

The envelope is, per converter fixture and path (loop / prefill / ppl), the largest
GPU-vs-oracle error any test saw; tests/bars.py sets each fixture bar to 8x it (capped by the
north-star bar).  Synthetic-model checks (fixture None) keep the north-star bar."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    log = json.load(open(sys.argv[1]))
    env = {}
    for _test, fixture, path, err, _scale in log:
        if fixture is None:
            continue
        d = env.setdefault(fixture, {})
        d[path] = max(d.get(path, 0.0), err)
    # a path with zero measured error (bit-identical) gets the float32 resolution of 1
    for d in env.values():
        for k, v in d.items():
            d[k] = max(v, 1.2e-7)
    out = os.path.join(ROOT, "tests", "golden", "error_envelope.json")
    with open(out, "w") as f:
        json.dump(dict(sorted(env.items())), f, indent=1, sort_keys=True)
    for k, v in sorted(env.items()):
        print(k, {p: f"{e:.3g}" for p, e in v.items()})


if __name__ == "__main__":
    main()
