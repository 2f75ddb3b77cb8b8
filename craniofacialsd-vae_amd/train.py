"""Training driver: ``train.py`` of the reference (train.py:13-80) on the
libcfsd path.  Same CLI (``--config --id --output_path --resume``) and YAML
schema (configurations/craniofacial.yaml: data / optimization / model /
logging_frequency), plus ``--precision`` and ``--no-graph``.  Launched by
``torch.distributed.run`` with N processes it trains data-parallel (one GPU
per rank, each rank on its shard of the training set, RCCL all-reduce of the
gradient, rank 0 logging and checkpointing).

Per epoch: a training pass and a no-grad validation pass over resident,
device-shuffled, device-swapped batches (model_manager.py:257-272), the
per-epoch loss means logged (model_manager.py:575-592; JSON lines under
``<output>/logs``), checkpoints every ``logging_frequency.save_weights``
epochs in the reference's ``model_%08d.pt`` / ``optimizer.pt`` format.  At the
end the latent statistics of the training set (test.py:95-117) are saved.
Rendering (tb_renderings), latent traversal videos and the classifiers are
out of scope.
"""
import argparse
import os
import shutil
import sys
import time


def main(argv=None):
    parser = argparse.ArgumentParser()
    parser.add_argument("--config", type=str, default="configurations/default.yaml",
                        help="Path to the configuration file.")
    parser.add_argument("--id", type=str, default="none", help="ID of experiment")
    parser.add_argument("--output_path", type=str, default=".", help="outputs path")
    parser.add_argument("--resume", action="store_true")
    parser.add_argument("--precision", default="fp32", choices=["fp32", "bf16"])
    parser.add_argument("--no-graph", action="store_true", help="eager launches (no hipGraph replay)")
    parser.add_argument("--epochs", type=int, default=None, help="override optimization.epochs")
    parser.add_argument("--seed", type=int, default=0)
    opts = parser.parse_args(argv)

    import torch

    from . import data as D
    from . import dist as DD
    from . import manager as M

    # data parallel under torchrun (configuration C3): one process per GPU,
    # RCCL gradient all-reduce; rank 0 writes logs, checkpoints and stats
    world, rank, local = DD.env_world()
    if os.environ.get("CFSD_SHARE_DEVICE"):  # rehearsal: all ranks on GPU 0 (tests, gloo)
        local = 0
    if not torch.cuda.is_available():
        raise RuntimeError("craniofacialsd_vae_amd trains on the GPU only (libcfsd); no GPU visible")
    device = torch.device("cuda", local if world > 1 else torch.cuda.current_device())
    torch.cuda.set_device(device)
    averager = None
    if world > 1:
        DD.init_from_env(backend=os.environ.get("CFSD_DIST_BACKEND", "nccl"), device_id=device)
        averager = DD.GradientAverager(world)
    lead = rank == 0

    config = M.load_config(opts.config)
    model_name = opts.id if opts.id != "none" else os.path.splitext(os.path.basename(opts.config))[0]
    output_directory = os.path.join(opts.output_path + "/outputs", model_name)
    checkpoint_dir = M.prepare_sub_folder(output_directory)
    writer = M.JsonlWriter(os.path.join(output_directory, "logs")) if lead else None
    if lead:
        shutil.copy(opts.config, os.path.join(output_directory, "config.yaml"))

    manager = M.ModelManager(config, device=device,
                             precomputed_storage_path=config["data"]["precomputed_path"],
                             precision=opts.precision, seed=opts.seed + rank, use_graph=not opts.no_graph,
                             averager=averager)
    bs = config["optimization"]["batch_size"]
    if world > 1:  # the split / augmentation / norm files are made once, by rank 0
        if lead:
            D.prepare_split(config["data"], manager.template, device, opts.seed)
        DD.barrier()
    train_set, val_set, test_set, norm = D.load_mesh_dataset(config["data"], bs, device, manager.template,
                                                             shard=(rank, world), seed=opts.seed)
    start_epoch = manager.resume(checkpoint_dir) if opts.resume else 0
    epochs = opts.epochs if opts.epochs is not None else config["optimization"]["epochs"]
    save_every = config.get("logging_frequency", {}).get("save_weights", 100)
    history = []
    for epoch in range(start_epoch, epochs):
        t0 = time.perf_counter()
        tr = manager.run_epoch(train_set, train=True)
        va = manager.run_epoch(val_set, train=False) if val_set is not None else None
        history.append({"epoch": epoch + 1, "train": tr, "validation": va,
                        "seconds": time.perf_counter() - t0})
        if lead:
            manager.log_losses(writer, epoch, "train", tr)
            if va is not None:
                manager.log_losses(writer, epoch, "validation", va)
            print(f"epoch {epoch + 1}: train tot {tr['tot']:.5f}"
                  + (f", validation tot {va['tot']:.5f}" if va else ""), flush=True)
            if (epoch + 1) % save_every == 0:
                manager.save_weights(checkpoint_dir, epoch)
    # latent statistics of the training set (Tester.compute_latent_stats)
    if lead:
        z = manager.encode(train_set.meshes)
        stats = manager.engine.latent_stats(z)
        torch.save({k: v.cpu() for k, v in stats.items()}, os.path.join(output_directory, "z_stats.pt"))
    if world > 1:
        DD.barrier()
        DD.destroy()
    return manager, history


if __name__ == "__main__":
    sys.exit(0 if main() else 1)
