"""MI355X-native ticker<->news keyword matching (drop-in for match_keywords.py).

Modules:
  kb             knowledge-base loading / classification / pattern compile (host)
  matcher        arena packing, the libkwmatch GPU handle, result assembly
  match_keywords the drop-in replacement of the reference script
  dedup          CDX URL keep-first dedup on the GPU
  dist           multi-GPU sharding + RCCL gather of hit records
  synth          seeded synthetic corpus (bench/test data)
"""
__all__ = ['kb', 'matcher', 'match_keywords']
