"""One rank of the engine's multi-rank campaign (tests/test_distributed.py::
test_engine_two_ranks_one_gpu): FaultCampaign.run(num_gpus=WORLD_SIZE) over
gloo with every rank on device 0; writes its outcomes and the reduced
histogram under OUTDIR.  Started as a plain child process by the test."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch.distributed as dist
    from shrewd_amd.fi import FaultCampaign
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    outdir, trials, seed = sys.argv[1], int(sys.argv[2]), int(sys.argv[3], 0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fc = FaultCampaign(os.path.join(ROOT, "workloads", "crc32.elf"), cmd=["crc32"], trials=trials, seed=seed,
                           structures=("int_reg", "pc"), num_gpus=world, device=0)
        out = fc.run()
        np.save(os.path.join(outdir, f"out{rank}.npy"), out)
        h = fc.histogram()
        np.save(os.path.join(outdir, f"hist{rank}.npy"), np.frombuffer(h.tobytes(), np.uint8))
        with open(os.path.join(outdir, f"first{rank}.txt"), "w") as f:
            f.write(str(fc.first))
        fc.engine.close()
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
