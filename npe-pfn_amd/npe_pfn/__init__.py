"""MI355X-native NPE-PFN (package name kept from the reference for drop-in use)."""
