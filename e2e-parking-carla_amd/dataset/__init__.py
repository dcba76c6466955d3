"""Reference dataset/ package: CarlaDataset, ParkingDataModule and the MI355X frame cache."""
