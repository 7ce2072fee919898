"""cylon_amd.parallel"""
