"""Writes a synthetic pre-tokenized corpus (memory-map format) for the examples (args: prefix, #docs, vocab):
documents of random length with ids drawn from a Zipf-like distribution, each ended by EOS id 0."""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from scaling_amd.core import MemoryMapDatasetBuilder  # noqa: E402

if __name__ == "__main__":
    prefix = Path(sys.argv[1] if len(sys.argv) > 1 else "examples/transformer_example/data/data")
    n_docs = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    vocab = int(sys.argv[3]) if len(sys.argv) > 3 else 128000
    rng = np.random.RandomState(0)
    if Path(str(prefix) + ".meta.json").exists():
        print(f"{prefix} exists")
        sys.exit(0)
    prefix.parent.mkdir(parents=True, exist_ok=True)
    with MemoryMapDatasetBuilder(prefix) as b:
        for _ in range(n_docs):
            n = int(rng.randint(16, 512))
            b.add(np.concatenate([np.minimum(rng.zipf(1.3, size=n), vocab - 1), [0]]).astype(np.int32))
    print(f"wrote {n_docs} documents to {prefix}")
