"""cylon_amd.indexing"""
