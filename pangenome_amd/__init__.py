"""MI355X-native build of Rinoahu/pangenome's k-mer -> dBG -> rdBG -> region-table path.

The compute runs in libpangenome_hip.so (HIP, gfx950); see include/pangenome.h
for the C ABI and pangenome_amd.kmer for the reference-compatible interface.
"""
__all__ = ["kmer", "host", "synth"]
