"""Human-friendly random names for identifiers without an explicit ``name``.

The reference uses ``golang-petname`` (``identifier.go:61-75``): ``adverb-adjective-name``.
The word lists here are our own; only the shape (N dash-separated lowercase words) matters
for compatibility because random identifiers are never re-derived.
"""
from __future__ import annotations

import os


def _choice(seq):
    """``secrets.choice`` without importing ``secrets`` (it pulls in hmac/OpenSSL: ~4 ms of
    every CLI start); the same OS randomness."""
    n = len(seq)
    limit = (1 << 32) - (1 << 32) % n  # rejection sampling: no modulo bias
    while True:
        x = int.from_bytes(os.urandom(4), "little")
        if x < limit:
            return seq[x % n]


ADVERBS = (
    "ably", "aptly", "boldly", "briskly", "calmly", "deftly", "eagerly", "evenly",
    "fairly", "firmly", "freely", "gently", "gladly", "keenly", "kindly", "lively",
    "loudly", "neatly", "nicely", "openly", "proudly", "quickly", "quietly", "rapidly",
    "really", "safely", "sharply", "simply", "smoothly", "solely", "steadily", "surely",
    "swiftly", "tightly", "truly", "vastly", "warmly", "wisely",
)
ADJECTIVES = (
    "able", "amber", "bold", "brave", "bright", "calm", "clever", "cosmic", "crisp",
    "dapper", "eager", "epic", "fast", "fine", "fluent", "fresh", "giant", "golden",
    "grand", "happy", "humble", "ideal", "jolly", "keen", "large", "lucid", "lucky",
    "mellow", "mighty", "modest", "noble", "polite", "quick", "rapid", "ready", "sharp",
    "silent", "smart", "solid", "steady", "sunny", "swift", "tidy", "vivid", "witty",
)
NAMES = (
    "albatross", "antelope", "badger", "beaver", "bison", "bobcat", "buffalo", "camel",
    "cheetah", "condor", "coyote", "crane", "dingo", "dolphin", "eagle", "falcon",
    "ferret", "finch", "gazelle", "gecko", "gopher", "heron", "hornet", "ibex", "impala",
    "jaguar", "kestrel", "koala", "lemur", "lynx", "marmot", "meerkat", "mongoose",
    "narwhal", "ocelot", "osprey", "otter", "panther", "pelican", "puffin", "quail",
    "raven", "salmon", "seal", "sparrow", "tapir", "toucan", "walrus", "wombat", "zebra",
)


def generate(words: int = 3, separator: str = "-") -> str:
    if words <= 0:
        return ""
    parts = [_choice(NAMES)]
    if words >= 2:
        parts.insert(0, _choice(ADJECTIVES))
    for _ in range(words - 2):
        parts.insert(0, _choice(ADVERBS))
    return separator.join(parts)
