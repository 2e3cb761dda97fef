"""Drop-in mirrors of the reference's ``model/`` classes (SoraKurihara/FFM)."""
