import os

if __name__ == "__main__":
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:     # launched by torch.distributed.run: one rank per GPU
        from .dist import main
    else:
        from .kmer import main
    raise SystemExit(main())
