"""MI355X-native per-family duplex consensus hot path (drop-in for
DuplexUMIConsensusReads.make_consensus_read and its callers)."""

__all__ = ["records", "bam"]
