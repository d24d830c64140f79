"""quest_amd.ops"""
