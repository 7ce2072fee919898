"""cylon_amd.utils"""
