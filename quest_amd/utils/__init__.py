"""quest_amd.utils"""
