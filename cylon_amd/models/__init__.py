"""cylon_amd.models"""
