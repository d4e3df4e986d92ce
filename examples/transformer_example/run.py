"""python -m examples.transformer_example.run examples/transformer_example/config.yml"""
import argparse

from scaling_amd.core import runner_main
from scaling_amd.core.logging import logger
from scaling_amd.transformer import TransformerConfig

if __name__ == "__main__":
    parser = argparse.ArgumentParser()
    parser.add_argument("config", type=str)
    args = parser.parse_args()
    config = TransformerConfig.from_yaml(args.config)
    logger.configure(config=config.logger, name="runner")
    runner_main(config.runner, payload=config.as_dict())
