"""GPU diagnostics: one FusedStep per production fixture, printing the
relative error of every checked quantity instead of asserting."""
import sys

import torch

sys.path.insert(0, "tests")
from golden_io import PROD, load_prod, prod_inputs  # noqa: E402
from gpu_helpers import rel_err  # noqa: E402
from test_prod_fixtures import build_product  # noqa: E402


def main(names):
    from modules import engine, noise
    for name in names or PROD:
        meta, arr = load_prod(name)
        enc, samp, dec = build_product(meta, "cuda")
        step = engine.FusedStep(enc, samp, dec)
        inp = prod_inputs(meta)
        q = [] if inp["feat_noise"] is None else [inp["feat_noise"]]
        noise.replay(*(q + [inp["eps"]]))
        sc, logits = step.forward_backward(inp["data"].cuda(), inp["batch_sizes"], inp["is_offset"].cuda(),
                                           inp["speakers"].cuda(), meta["N"], is_pretraining=meta.get("pretrain", False))
        torch.cuda.synchronize()
        sc = sc.cpu()
        out = {k: (float(sc[i]) - float(arr[k])) / abs(float(arr[k]))
               for i, k in ((engine.EM, "em"), (engine.OFF, "off"), (engine.KL, "kl"), (engine.LOSS, "loss"))}
        out["hidden"] = rel_err(step.last_hidden, arr["last_hidden"])
        out["logits"] = rel_err(logits, arr["logits"])
        out["feats"] = rel_err(step.feats, arr["feats"])
        print(name, {k: "%.2e" % v for k, v in out.items()}, flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
