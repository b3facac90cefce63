"""Host-side mirrors of the reference ``utils`` package (consensus engines and weight design)."""
