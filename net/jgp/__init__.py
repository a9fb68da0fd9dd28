"""Namespace scaffolding mirroring the reference Java package net.jgp.labs."""
