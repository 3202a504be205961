"""``python -m infrared-colorization-with-resnet-generator-and-patchgan_amd [train|test]``
-- the reference's script entry point (ir:1730-1756) with cfg.mode taken from
the command line (default: Config's "test")."""
import sys

from .ir_colorization import Config, main

if __name__ == "__main__":
    cfg = Config()
    if len(sys.argv) > 1:
        cfg.mode = sys.argv[1]
    main(cfg)
