"""Model families with the reference ``src/models`` API (UNets + factory)."""
