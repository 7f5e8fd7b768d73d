"""TEST HARNESS (not product code): a pure-Python host path over the oracle
backends — per-family preprocessing (pipeline.py), a record writer over the
AlignedSegment stand-in (writer.py) and chunked multi-rank sharding
(shard.py).  The product path is duplexumiconsensusreads_amd.cli over the
native ingest, the device stream and the native / device writers; the tests
use this harness as an independent restatement to check those against."""
